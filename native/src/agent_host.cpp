// Agent: what it changes on the host besides addresses, and puts back -- the stale label and
// the networkd directory at start, NIC-firmware LLDP / DCBX (--disable-fw-lldp and its state
// file), the NICs' MTUs (--restore-mtu / --mtu-state), NetworkManager, and the teardown on exit.
#include "netop/agent.hpp"

#include <errno.h>
#include <linux/if.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cstddef>

#include <algorithm>
#include <cstring>
#include <ctime>
#include <sched.h>
#include <sys/syscall.h>
#include <mutex>
#include <regex>
#include <set>
#include <system_error>

#include "agent_internal.hpp"
#include "netop/log.hpp"

namespace netop::agent {

using detail::fd_readable;

void Agent::pre_cleanups() {
    // Stale label from a previous (crashed) run: the node is not ready until we say so.
    if (path_exists(cfg_.labels.path())) {
        NLOG_I("NFD label file already exists, removing it...");
        if (!artifacts::remove_labels(cfg_.labels)) NLOG_W("Failed to remove NFD label file: %s", std::strerror(errno));
    }
    if (!cfg_.networkd.empty()) {
        try {
            mkdir_p(cfg_.networkd);
        } catch (const std::exception& e) {
            throw AgentError(std::string("Failed to pre-cleanup: Cannot create systemd-networkd directory: ") + e.what());
        }
        NLOG_I("Created systemd-networkd directory %s", cfg_.networkd.c_str());
    }
}

void Agent::disable_fw_lldp() {
    std::vector<ethtool::FlagRule> rules;
    try {
        rules = ethtool::parse_rules(cfg_.fw_lldp_flags);
    } catch (const std::exception& e) {
        throw AgentError(std::string("Invalid --fw-lldp-priv-flag: ") + e.what());
    }
    if (!ethtool_) {
        try {
            ethtool_ = ethtool::make_ioctl_ops();
        } catch (const std::exception& e) {
            NLOG_W("ethtool unavailable, firmware LLDP agents left alone: %s", e.what());
            return;
        }
    }
    // An earlier agent of this node (--keep-config) may have changed them already: its record
    // holds the real originals, which this run must neither lose nor take for "already set".
    // (Read without --keep-config too: an agent that failed left them changed, or the policy just
    // dropped keepConfigOnRestart; this agent then restores the true originals on a clean exit.)
    std::map<std::string, ethtool::FwLldpResult> earlier;
    if (!cfg_.fw_lldp_state.empty())
        if (auto t = read_file(cfg_.fw_lldp_state))
            for (auto& e : ethtool::decode_state(*t)) earlier[e.ifname] = e;
    for (auto& n : nics_) {
        auto r = ethtool::disable_fw_lldp(*ethtool_, n.ifname, rules, true, cfg_.fw_lldp_dcbx_host);
        n.fw_lldp = r.summary();
        if (r.dcbx) n.dcbx = ethtool::dcbx_str(*r.dcbx);
        n.dcbx_embedded = r.dcbx && ethtool::dcbx_embedded(*r.dcbx) && !r.dcbx_changed;
        if (!r.error.empty()) NLOG_W("%s: firmware LLDP: %s", n.ifname.c_str(), r.error.c_str());
        NLOG_V(2, "%s: driver %s, firmware LLDP: %s", n.ifname.c_str(), r.driver.c_str(), n.fw_lldp.c_str());
        if (auto it = earlier.find(n.ifname); it != earlier.end()) {
            if (it->second.changed) {
                r.changed = true;
                r.original_bits = it->second.original_bits;
            }
            if (it->second.dcbx_changed) {
                r.dcbx_changed = true;
                r.dcbx = it->second.dcbx;
            }
            earlier.erase(it);
        }
        fw_lldp_.push_back(std::move(r));
    }
    // What is left of the record belongs to NICs this agent does not select any more: they are
    // not ours now, so their originals go back at once; one that cannot be reached (renamed,
    // gone) stays in the record for --cleanup.
    for (auto& [name, r] : earlier) {
        NLOG_I("%s: no longer selected; restoring its firmware LLDP settings", name.c_str());
        if (!ethtool::restore(*ethtool_, r)) fw_lldp_carried_.push_back(r);
    }
    save_fw_lldp_state();
}

void Agent::save_fw_lldp_state(bool with_current) {
    if (cfg_.fw_lldp_state.empty()) return;  // also without --keep-config: an agent that fails leaves them changed
    try {
        std::vector<ethtool::FwLldpResult> all;
        if (with_current) all = fw_lldp_;
        all.insert(all.end(), fw_lldp_carried_.begin(), fw_lldp_carried_.end());
        const std::string text = ethtool::encode_state(all);
        if (!text.empty())
            write_file_atomic(cfg_.fw_lldp_state, text);
        else if (::unlink(cfg_.fw_lldp_state.c_str()) != 0 && errno != ENOENT)
            NLOG_W("Could not remove %s: %s", cfg_.fw_lldp_state.c_str(), std::strerror(errno));
    } catch (const std::exception& e) {
        NLOG_W("Could not record the firmware LLDP originals in %s: %s", cfg_.fw_lldp_state.c_str(), e.what());
    }
}

void Agent::restore_fw_lldp_from_state() {
    // --cleanup: what --keep-config agents changed on this node's NICs, from their record.
    if (cfg_.fw_lldp_state.empty()) return;
    auto t = read_file(cfg_.fw_lldp_state);
    if (!t) return;
    auto recs = ethtool::decode_state(*t);
    if (!recs.empty() && !ethtool_) ethtool_ = ethtool::make_ioctl_ops();
    for (const auto& r : recs) {
        NLOG_I("%s: restoring the NIC's firmware LLDP settings%s%s", r.ifname.c_str(),
               r.changed ? strfmt(" (private flags 0x%x)", r.original_bits).c_str() : "",
               r.dcbx_changed ? (" (DCBX " + ethtool::dcbx_str(*r.dcbx) + ")").c_str() : "");
        ethtool::restore(*ethtool_, r);
    }
    if (::unlink(cfg_.fw_lldp_state.c_str()) != 0 && errno != ENOENT)
        NLOG_W("Could not remove %s: %s", cfg_.fw_lldp_state.c_str(), std::strerror(errno));
}

void Agent::post_cleanups() {
    NLOG_I("Clean up before exiting...");
    if (ethtool_ && !persist_fw_lldp()) {  // kept on the node for the next agent / --cleanup otherwise
        for (const auto& r : fw_lldp_) ethtool::restore(*ethtool_, r);
        if (!fw_lldp_.empty()) save_fw_lldp_state(false);  // only what could not be reached stays (normally: none)
    }
    if (cfg_.lldp_announce && cfg_.mode == "L3" && !cfg_.keep_config) {
        // Shutdown LLDPDU (TTL 0): the switch drops us from its neighbour table right away.
        for (auto& n : nics_) {
            if (!n.link.up()) continue;
            try {
                lldp_->announce(n.ifname, lldp::encode(make_node_frame(cfg_.node_name, n.ifname, n.link.mac, n.gpu_bdf, 0)));
            } catch (...) {
            }
        }
    }
    if (!artifacts::remove_labels(cfg_.labels)) NLOG_W("Failed to remove NFD label file: %s", std::strerror(errno));
    if (cfg_.keep_config) {
        // The next agent adopts addresses, routes and rail rules; jobs keep their links meanwhile.
        NLOG_I("Keeping addresses, routes and links for the next agent (--keep-config)");
        return;
    }
    NLOG_I("Restoring interfaces to original state...");
    remove_rail_routing();
    try {
        remove_existing_ips();
    } catch (const std::exception& e) {
        NLOG_W("Failed to remove any existing IPs from interfaces: %s", e.what());
    }
    if (cfg_.restore_mtu) restore_mtus();
    try {
        interfaces_restore_down();
    } catch (const std::exception& e) {
        NLOG_W("Failed to restore interfaces to original state: %s", e.what());
    }
    restore_network_manager();
}

namespace {
std::map<std::string, int> read_mtu_state(const std::string& path) {
    std::map<std::string, int> out;
    auto t = read_file(path);
    if (!t) return out;
    for (const auto& line : split(*t, '\n')) {
        auto f = split(trim(line), ' ');
        if (f.size() != 2 || f[0].empty() || f[0].size() > 15) continue;
        try {
            const int mtu = std::stoi(f[1]);
            if (mtu >= 68 && mtu <= 65535) out[f[0]] = mtu;
        } catch (const std::exception&) {
        }
    }
    return out;
}

void write_mtu_state(const std::string& path, const std::map<std::string, int>& m) {
    if (m.empty()) {
        if (::unlink(path.c_str()) != 0 && errno != ENOENT)
            NLOG_W("Could not remove %s: %s", path.c_str(), std::strerror(errno));
        return;
    }
    std::string t;
    for (const auto& [n, mtu] : m) t += n + " " + std::to_string(mtu) + "\n";
    write_file_atomic(path, t);
}
}  // namespace

void Agent::load_mtu_state() {
    // The first agent's view of each NIC is the original; a later (--keep-config) agent finds the
    // MTU it set itself, so the recorded value wins.
    if (!cfg_.restore_mtu || cfg_.mtu_state.empty()) return;
    auto m = read_mtu_state(cfg_.mtu_state);
    for (auto& n : nics_) {
        auto it = m.find(n.ifname);
        if (it == m.end())
            m[n.ifname] = n.orig_mtu;
        else
            n.orig_mtu = it->second;
    }
    try {
        write_mtu_state(cfg_.mtu_state, m);
    } catch (const std::exception& e) {
        NLOG_W("Could not record the NICs' MTUs in %s: %s", cfg_.mtu_state.c_str(), e.what());
    }
}

void Agent::restore_mtus() {
    // Host NICs are the node's general-purpose interfaces: the MTU they had goes back with the
    // agent (the reference, and amd-so, leave the scale-out rails at the policy's MTU).
    std::map<std::string, int> left = cfg_.mtu_state.empty() ? std::map<std::string, int>{}
                                                              : read_mtu_state(cfg_.mtu_state);
    for (auto& n : nics_) {
        if (n.orig_mtu <= 0) continue;
        bool ok = n.link.mtu == n.orig_mtu;
        if (!ok) {
            try {
                ops_.link_set_mtu(n.link.index, n.orig_mtu);
                NLOG_I("Setting MTU of '%s' back to %d", n.ifname.c_str(), n.orig_mtu);
                n.link.mtu = n.orig_mtu;
                ok = true;
            } catch (const std::exception& e) {
                NLOG_W("Cannot set MTU of '%s' back to %d: %s", n.ifname.c_str(), n.orig_mtu, e.what());
            }
        }
        if (ok) left.erase(n.ifname);
    }
    if (!cfg_.mtu_state.empty()) {
        try {
            write_mtu_state(cfg_.mtu_state, left);  // what could not be put back stays for --cleanup
        } catch (const std::exception& e) {
            NLOG_W("Could not update %s: %s", cfg_.mtu_state.c_str(), e.what());
        }
    }
}

void Agent::restore_mtu_state() {
    if (!cfg_.restore_mtu || cfg_.mtu_state.empty()) return;
    auto m = read_mtu_state(cfg_.mtu_state);
    std::map<std::string, int> left;
    for (const auto& [name, mtu] : m) {
        try {
            auto l = ops_.link_by_name(name);
            if (l.mtu != mtu) {
                ops_.link_set_mtu(l.index, mtu);
                NLOG_I("Setting MTU of '%s' back to %d", name.c_str(), mtu);
            }
        } catch (const std::exception& e) {
            NLOG_W("Cannot set MTU of '%s' back to %d: %s", name.c_str(), mtu, e.what());
            left[name] = mtu;
        }
    }
    write_mtu_state(cfg_.mtu_state, left);
}

namespace {
std::map<std::string, bool> read_link_state(const std::string& path) {
    std::map<std::string, bool> out;
    auto t = read_file(path);
    if (!t) return out;
    for (const auto& line : split(*t, '\n')) {
        auto f = split(trim(line), ' ');
        if (f.size() != 2 || f[0].empty() || f[0].size() > 15 || (f[1] != "up" && f[1] != "down")) continue;
        out[f[0]] = f[1] == "up";
    }
    return out;
}

void write_link_state(const std::string& path, const std::map<std::string, bool>& m) {
    if (m.empty()) {
        if (::unlink(path.c_str()) != 0 && errno != ENOENT)
            NLOG_W("Could not remove %s: %s", path.c_str(), std::strerror(errno));
        return;
    }
    std::string t;
    for (const auto& [n, up] : m) t += n + (up ? " up\n" : " down\n");
    write_file_atomic(path, t);
}
}  // namespace

void Agent::load_link_state() {
    // Before interfaces_up(): the first agent records what it found; a later one (after a crash or
    // a --keep-config restart) finds the links up, and the record wins.
    if (cfg_.link_state.empty()) return;
    auto m = read_link_state(cfg_.link_state);
    for (auto& n : nics_) {
        auto it = m.find(n.ifname);
        if (it == m.end())
            m[n.ifname] = (n.orig_flags & IFF_UP) != 0;
        else if (it->second)
            n.orig_flags |= IFF_UP;
        else
            n.orig_flags &= ~unsigned(IFF_UP);
    }
    try {
        write_link_state(cfg_.link_state, m);
    } catch (const std::exception& e) {
        NLOG_W("Could not record the NICs' link states in %s: %s", cfg_.link_state.c_str(), e.what());
    }
}

void Agent::forget_link_state() {
    if (cfg_.link_state.empty()) return;
    auto m = read_link_state(cfg_.link_state);
    for (const auto& n : nics_)
        if (n.link.up() == ((n.orig_flags & IFF_UP) != 0)) m.erase(n.ifname);  // what failed stays for --cleanup
    try {
        write_link_state(cfg_.link_state, m);
    } catch (const std::exception& e) {
        NLOG_W("Could not update %s: %s", cfg_.link_state.c_str(), e.what());
    }
}

void Agent::restore_link_state() {
    if (cfg_.link_state.empty()) return;
    std::map<std::string, bool> left;
    for (const auto& [name, up] : read_link_state(cfg_.link_state)) {
        if (up) continue;  // it was up before any agent: it stays up
        try {
            auto l = ops_.link_by_name(name);
            if (l.up()) {
                ops_.link_set_down(l.index);
                NLOG_I("Setting link '%s' back down", name.c_str());
            }
        } catch (const SysError& e) {
            if (e.code() == ENODEV) continue;  // the NIC is gone
            NLOG_W("Cannot set link '%s' back down: %s", name.c_str(), e.what());
            left[name] = up;
        } catch (const std::exception& e) {
            NLOG_W("Cannot set link '%s' back down: %s", name.c_str(), e.what());
            left[name] = up;
        }
    }
    write_link_state(cfg_.link_state, left);
}

void Agent::restore_network_manager() {
    // Only with --nm-restore: the reference leaves its runtime Managed=false behind, and this
    // agent's keyfile keeps the NICs unmanaged across agent restarts and reboots (Config::nm_restore).
    if (!cfg_.nm_restore) return;
    if (nm_keyfile_written_ && nm::remove_keyfile(cfg_.nm_keyfile_dir, nm::keyfile_name(cfg_.labels.file))) {
        NLOG_I("Removed NetworkManager keyfile from %s", cfg_.nm_keyfile_dir.c_str());
        nm_keyfile_written_ = false;
    }
    if (nm_unmanaged_.empty()) return;
    try {
        auto nmapi = nm_factory_();
        nm::restore_for_interfaces(*nmapi, nm_unmanaged_);
        nm_unmanaged_.clear();
    } catch (const std::exception& e) {
        NLOG_W("Could not hand the interfaces back to NetworkManager: %s", e.what());
    }
}

}  // namespace netop::agent
