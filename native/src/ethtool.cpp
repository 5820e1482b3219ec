#include "netop/ethtool.hpp"

#include <linux/dcbnl.h>
#include <linux/ethtool.h>
#include <linux/sockios.h>
#include <net/if.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "netop/common.hpp"
#include "netop/log.hpp"
#include "netop/netlink.hpp"

namespace netop::ethtool {

int PrivFlags::index_of(const std::string& name) const {
    for (size_t i = 0; i < names.size(); ++i)
        if (names[i] == name) return int(i);
    return -1;
}

namespace {

class IoctlOps final : public Ops {
   public:
    IoctlOps() : fd_(::socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0)) {
        if (fd_ < 0) throw SysError(errno, "ethtool socket");
    }
    ~IoctlOps() override { ::close(fd_); }

    std::string driver(const std::string& ifname) override {
        ethtool_drvinfo info{};
        info.cmd = ETHTOOL_GDRVINFO;
        if (!call(ifname, &info, false)) return "";
        return std::string(info.driver, strnlen(info.driver, sizeof info.driver));
    }

    PrivFlags get(const std::string& ifname) override {
        PrivFlags pf;
        // Number of private-flag strings: ETHTOOL_GSSET_INFO with the PRIV_FLAGS bit.
        alignas(8) uint8_t ssbuf[sizeof(ethtool_sset_info) + sizeof(uint32_t)] = {};
        auto* ss = reinterpret_cast<ethtool_sset_info*>(ssbuf);
        ss->cmd = ETHTOOL_GSSET_INFO;
        ss->sset_mask = 1ull << ETH_SS_PRIV_FLAGS;
        call(ifname, ss, true);
        uint32_t n = 0;
        if (ss->sset_mask & (1ull << ETH_SS_PRIV_FLAGS)) std::memcpy(&n, ssbuf + sizeof(ethtool_sset_info), sizeof n);
        if (n == 0) return pf;
        if (n > 32) n = 32;  // the flags word is 32 bits wide
        std::vector<uint8_t> buf(sizeof(ethtool_gstrings) + size_t(n) * ETH_GSTRING_LEN);
        auto* gs = reinterpret_cast<ethtool_gstrings*>(buf.data());
        gs->cmd = ETHTOOL_GSTRINGS;
        gs->string_set = ETH_SS_PRIV_FLAGS;
        gs->len = n;
        call(ifname, gs, true);
        for (uint32_t i = 0; i < gs->len && i < n; ++i) {
            const char* s = reinterpret_cast<const char*>(gs->data) + size_t(i) * ETH_GSTRING_LEN;
            pf.names.emplace_back(s, strnlen(s, ETH_GSTRING_LEN));
        }
        ethtool_value v{};
        v.cmd = ETHTOOL_GPFLAGS;
        call(ifname, &v, true);
        pf.bits = v.data;
        return pf;
    }

    void set(const std::string& ifname, uint32_t bits) override {
        ethtool_value v{};
        v.cmd = ETHTOOL_SPFLAGS;
        v.data = bits;
        call(ifname, &v, true);
    }

    std::optional<uint8_t> dcbx_get(const std::string& ifname) override { return rtnl().dcbx_mode(ifname); }
    bool dcbx_set(const std::string& ifname, uint8_t mode) override { return rtnl().set_dcbx_mode(ifname, mode); }

   private:
    bool call(const std::string& ifname, void* data, bool throw_on_error) {
        ifreq ifr{};
        if (ifname.size() >= IFNAMSIZ) throw SysError(EINVAL, "interface name too long: " + ifname);
        std::memcpy(ifr.ifr_name, ifname.c_str(), ifname.size());
        ifr.ifr_data = static_cast<char*>(data);
        if (::ioctl(fd_, SIOCETHTOOL, &ifr) == 0) return true;
        if (throw_on_error) throw SysError(errno, "SIOCETHTOOL " + ifname);
        return false;
    }
    nl::Rtnl& rtnl() {  // DCB netlink: a socket of its own, opened on first use
        if (!rtnl_) rtnl_ = std::make_unique<nl::Rtnl>();
        return *rtnl_;
    }
    int fd_;
    std::unique_ptr<nl::Rtnl> rtnl_;
};

}  // namespace

bool Ops::dcbx_set(const std::string& ifname, uint8_t mode) {
    (void)mode;
    throw SysError(EOPNOTSUPP, "DCB " + ifname);
}

std::string dcbx_str(uint8_t mode) {
    std::vector<std::string> w;
    if (mode & DCB_CAP_DCBX_HOST) w.push_back("host");
    if (mode & DCB_CAP_DCBX_LLD_MANAGED) w.push_back("lld-managed");
    if (!(mode & (DCB_CAP_DCBX_HOST | DCB_CAP_DCBX_LLD_MANAGED))) w.push_back("firmware");
    if (mode & DCB_CAP_DCBX_VER_CEE) w.push_back("cee");
    if (mode & DCB_CAP_DCBX_VER_IEEE) w.push_back("ieee");
    if (mode & DCB_CAP_DCBX_STATIC) w.push_back("static");
    return strfmt("0x%02x (%s)", mode, join(w, ", ").c_str());
}

bool dcbx_embedded(uint8_t mode) { return !(mode & DCB_CAP_DCBX_HOST); }

std::unique_ptr<Ops> make_ioctl_ops() { return std::make_unique<IoctlOps>(); }

std::vector<FlagRule> builtin_rules() { return {{"disable-fw-lldp", true}, {"fw-lldp-agent", false}}; }

std::vector<FlagRule> parse_rules(const std::string& spec) {
    std::vector<FlagRule> out;
    for (const auto& item : split(spec, ',')) {
        std::string t = trim(item);
        if (t.empty()) continue;
        auto eq = t.find('=');
        if (eq == std::string::npos || eq == 0) throw std::invalid_argument("bad private-flag rule '" + t + "' (want NAME=0|1)");
        std::string v = trim(t.substr(eq + 1));
        for (auto& c : v) c = char(std::tolower(static_cast<unsigned char>(c)));
        FlagRule r{trim(t.substr(0, eq)), true};
        if (v == "1" || v == "on" || v == "true")
            r.value = true;
        else if (v == "0" || v == "off" || v == "false")
            r.value = false;
        else
            throw std::invalid_argument("bad private-flag value in '" + t + "'");
        out.push_back(r);
    }
    for (const auto& b : builtin_rules()) out.push_back(b);
    return out;
}

std::string FwLldpResult::summary() const {
    if (!error.empty()) return "error: " + error;
    if (dry_run && would_change)
        return flag.empty() ? "would hand DCBX to the host (now " + dcbx_str(*dcbx) + ")" : "would set " + flag;
    if (!flag.empty()) return (changed ? "set " : "already ") + flag;
    if (dcbx_changed) return "DCBX handed to the host (was " + dcbx_str(*dcbx) + ")";
    if (dcbx) return "no firmware LLDP flag; DCBX " + dcbx_str(*dcbx);
    return "no firmware LLDP flag";
}

FwLldpResult disable_fw_lldp(Ops& ops, const std::string& ifname, const std::vector<FlagRule>& rules, bool apply,
                             bool hand_dcbx) {
    FwLldpResult r;
    r.ifname = ifname;
    r.dry_run = !apply;
    try {
        r.driver = ops.driver(ifname);
        PrivFlags pf = ops.get(ifname);
        r.original_bits = pf.bits;
        for (const auto& rule : rules) {
            int i = pf.index_of(rule.name);
            if (i < 0) continue;
            r.flag = rule.name + (rule.value ? "=on" : "=off");
            uint32_t bit = 1u << i;
            uint32_t want = rule.value ? (pf.bits | bit) : (pf.bits & ~bit);
            if (want != pf.bits && !apply) {
                r.would_change = true;
            } else if (want != pf.bits) {
                ops.set(ifname, want);
                r.changed = true;
                NLOG_I("%s (%s): firmware LLDP agent off via private flag %s", ifname.c_str(), r.driver.c_str(),
                       r.flag.c_str());
            }
            break;
        }
    } catch (const SysError& e) {
        // EOPNOTSUPP: the driver has no private flags at all (veth, virtio, ...): nothing to do.
        if (e.code() != EOPNOTSUPP) r.error = e.what();
    } catch (const std::exception& e) {
        r.error = e.what();
    }
    if (!r.flag.empty() || !r.error.empty()) return r;
    // No private flag for this driver: is an embedded agent running DCBX (and LLDP) here?
    try {
        r.dcbx = ops.dcbx_get(ifname);
        if (hand_dcbx && r.dcbx && dcbx_embedded(*r.dcbx)) {
            uint8_t want = uint8_t(DCB_CAP_DCBX_HOST | (*r.dcbx & (DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE)));
            if (!(want & (DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE))) want |= DCB_CAP_DCBX_VER_IEEE;
            if (!apply) {
                r.would_change = true;
            } else if (ops.dcbx_set(ifname, want)) {
                r.dcbx_changed = true;
                NLOG_I("%s (%s): DCBX handed to the host (was %s), so the NIC's embedded agent no longer runs LLDP",
                       ifname.c_str(), r.driver.c_str(), dcbx_str(*r.dcbx).c_str());
            } else {
                r.error = "the driver refused DCBX host mode " + dcbx_str(want) + " (current " + dcbx_str(*r.dcbx) + ")";
            }
        }
    } catch (const std::exception& e) {
        r.error = std::string("DCBX: ") + e.what();
    }
    return r;
}

bool restore(Ops& ops, const FwLldpResult& r) {
    bool all = true;
    if (r.changed) {
        try {
            ops.set(r.ifname, r.original_bits);
        } catch (const std::exception& e) {
            NLOG_W("%s: could not restore private flags: %s", r.ifname.c_str(), e.what());
            all = false;
        }
    }
    if (r.dcbx_changed) {
        // The original mode first; mlx5_core takes only 0 as "back to firmware (auto)" control.
        try {
            bool ok = ops.dcbx_set(r.ifname, *r.dcbx);
            if (!ok && !(*r.dcbx & DCB_CAP_DCBX_LLD_MANAGED)) ok = ops.dcbx_set(r.ifname, 0);
            if (!ok) NLOG_W("%s: the driver refused to restore DCBX mode %s", r.ifname.c_str(), dcbx_str(*r.dcbx).c_str());
            all &= ok;
        } catch (const std::exception& e) {
            NLOG_W("%s: could not restore the DCBX mode: %s", r.ifname.c_str(), e.what());
            all = false;
        }
    }
    return all;
}

std::string encode_state(const std::vector<FwLldpResult>& rs) {
    std::string out;
    for (const auto& r : rs) {
        if (r.changed) out += strfmt("%s priv 0x%x\n", r.ifname.c_str(), r.original_bits);
        if (r.dcbx_changed && r.dcbx) out += strfmt("%s dcbx 0x%02x\n", r.ifname.c_str(), *r.dcbx);
    }
    return out;
}

// The kernel's dev_valid_name: 1..15 bytes, not "." or "..", no '/', ':' or whitespace (and, for a
// record written with %s, printable: a NUL would cut it short).
static bool valid_ifname(const std::string& n) {
    if (n.empty() || n.size() >= 16 || n == "." || n == "..") return false;
    for (unsigned char c : n)
        if (c <= 0x20 || c >= 0x7f || c == '/' || c == ':') return false;
    return true;
}

std::vector<FwLldpResult> decode_state(const std::string& text) {
    std::vector<FwLldpResult> out;
    auto find = [&](const std::string& ifname) -> FwLldpResult& {
        for (auto& r : out)
            if (r.ifname == ifname) return r;
        out.emplace_back();
        out.back().ifname = ifname;
        return out.back();
    };
    for (const auto& line : split(text, '\n')) {
        auto f = split(trim(line), ' ');
        if (f.size() != 3 || !valid_ifname(f[0])) continue;
        char* end = nullptr;
        errno = 0;
        unsigned long v = std::strtoul(f[2].c_str(), &end, 16);
        if (errno || !end || *end || f[2].empty()) continue;
        if (f[1] == "priv" && v <= 0xffffffffUL) {
            auto& r = find(f[0]);
            r.changed = true;
            r.original_bits = uint32_t(v);
        } else if (f[1] == "dcbx" && v <= 0xffUL) {
            auto& r = find(f[0]);
            r.dcbx_changed = true;
            r.dcbx = uint8_t(v);
        }
    }
    return out;
}

}  // namespace netop::ethtool
