// `netop-lldp-tx` — synthetic ToR switch for the netns harness.
//
// Plays the switch side of the reference's contract: every switch port advertises a Port
// Description "<tag> a.b.c.d/30" (reference README.md:19-25).  Models an IEEE 802.1AB-2009
// LLDP agent:
//   * periodic transmission every --interval (msgTxInterval, 30 s on real switches), with the
//     first frame at a random phase in [0, interval) when --phase=random (a switch that has
//     been running for a while), or immediately with --phase=zero;
//   * optional fast start (--fast-start): when an LLDPDU from a *new neighbour* arrives on a
//     port, the port transmits immediately and then --tx-fast-init frames at --fast-interval
//     (txFastInit = 4, msgFastTx = 1 s in the standard);
//   * --assign-ip puts the peer address of the Port Description on the switch port so the
//     node's /30 is actually reachable.
//
//   * --system-name may contain "{port}" (the port's position in the --port list), so one
//     process can play one leaf switch per rail; --port-system-name IFNAME=NAME overrides one
//     port's (a miscabled NIC in the rail-check tests).
//
//   netop-lldp-tx --port sw0='no-alert 10.200.0.2/30' --port sw1=... [--interval 30s]
//                 [--phase random|zero] [--fast-start] [--count N] [--assign-ip] [--seed S]
#include <signal.h>
#include <sys/epoll.h>
#include <unistd.h>

#include <cstdio>
#include <map>
#include <random>
#include <set>

#include "netop/cli.hpp"
#include "netop/l3.hpp"
#include "netop/lldp.hpp"
#include "netop/log.hpp"
#include "netop/netlink.hpp"
#include "netop/packet.hpp"

using namespace netop;

static volatile sig_atomic_t g_stop = 0;
static void on_sig(int) { g_stop = 1; }

int main(int argc, char** argv) {
    std::vector<std::pair<std::string, std::string>> ports;
    int64_t interval = 30LL * 1000000000, fast_interval = 1000000000LL;
    int count = 0, tx_fast_init = 4, ttl = 120, verbosity = 0, seed = 0;
    std::string sysname = "tor-synthetic", phase = "random", mtu_str;
    bool fast_start = false, assign_ip = false;

    cli::FlagSet fs("netop-lldp-tx");
    fs.add_func("port", true, [&](const std::string& v) {
        auto eq = v.find('=');
        if (eq == std::string::npos) throw std::invalid_argument("--port wants IFNAME=PORT_DESCRIPTION");
        ports.emplace_back(v.substr(0, eq), v.substr(eq + 1));
    }, "IFNAME=PORT_DESCRIPTION (repeatable)");
    std::vector<std::string> silent;
    fs.add_func("silent-port", true, [&](const std::string& v) { silent.push_back(v); },
                "IFNAME: a port that is up (the NIC has carrier) but never transmits LLDP (repeatable)");
    fs.add_duration("interval", &interval, "msgTxInterval");
    fs.add_string("phase", &phase, "first periodic frame: random (U[0,interval)) or zero");
    fs.add_bool("fast-start", &fast_start, "802.1AB-2009 fast transmission on new neighbours");
    fs.add_duration("fast-interval", &fast_interval, "msgFastTx");
    fs.add_int("tx-fast-init", &tx_fast_init, "txFastInit");
    fs.add_int("count", &count, "periodic frames per port before exiting (0 = until SIGTERM)");
    fs.add_string("system-name", &sysname, "System Name TLV (\"{port}\" = the port's index)");
    std::map<std::string, std::string> port_sysname;
    fs.add_func("port-system-name", true, [&](const std::string& v) {
        auto eq = v.find('=');
        if (eq == std::string::npos) throw std::invalid_argument("--port-system-name wants IFNAME=NAME");
        port_sysname[v.substr(0, eq)] = v.substr(eq + 1);
    }, "IFNAME=NAME: this port's System Name (repeatable)");
    fs.add_int("ttl", &ttl, "TTL TLV");
    int max_frame = 0;
    fs.add_int("max-frame-size", &max_frame, "IEEE 802.3 Maximum Frame Size TLV (bytes; 0 = not sent)");
    fs.add_bool("assign-ip", &assign_ip, "assign the Port Description address to the switch port");
    fs.add_int("seed", &seed, "RNG seed for the random phase (0 = time based)");
    fs.add_int("v", &verbosity, "log verbosity");
    try {
        fs.parse(argc, argv);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error: %s\n%s", e.what(), fs.usage().c_str());
        return 2;
    }
    log::set_verbosity(verbosity);
    if (ports.empty() && silent.empty()) {
        std::fprintf(stderr, "Error: no --port given\n");
        return 2;
    }
    signal(SIGTERM, on_sig);
    signal(SIGINT, on_sig);
    std::mt19937_64 rng(seed ? uint64_t(seed) : uint64_t(wall_ns()));

    struct Port {
        std::unique_ptr<pkt::LldpSocket> sock;
        std::vector<uint8_t> frame;
        int64_t next = 0;
        int fast_left = 0;
        int periodic_sent = 0;
        std::set<std::string> neighbours;
    };
    std::vector<Port> ps;
    int ep = ::epoll_create1(EPOLL_CLOEXEC);
    std::unique_ptr<nl::Rtnl> rtnl_holder;
    // Bring a port up (and give it the switch side of its /30): at start, and again when the port
    // was re-created (the peer NIC's driver reload in the end-to-end harness).
    auto open_port = [&](nl::Rtnl& rtnl, const std::string& ifname, const std::string& desc, Port& p) {
        auto link = rtnl.link_by_name(ifname);
        if (!link.up()) rtnl.link_set_up(link.index);
        if (assign_ip) {
            if (auto a = l3::parse_port_description(desc, l3::TokenPolicy::CompatThenLast, nullptr)) {
                try {
                    rtnl.addr_add(link.index, Ipv4Prefix{a->peer, a->prefix});
                } catch (const SysError& e) {
                    if (e.code() != EEXIST) throw;
                }
            }
        }
        p.sock = std::make_unique<pkt::LldpSocket>(ifname, link.index, link.mac, false);
        std::string name = sysname;
        if (auto it = port_sysname.find(ifname); it != port_sysname.end()) {
            name = it->second;
        } else if (auto at = name.find("{port}"); at != std::string::npos) {
            size_t idx = 0;
            while (idx < ports.size() && ports[idx].first != ifname) ++idx;
            name.replace(at, 6, std::to_string(idx));
        }
        auto frame = lldp::make_switch_frame(link.mac, name, ifname, desc, uint16_t(ttl));
        if (max_frame > 0) frame.set_max_frame_size(uint16_t(max_frame));
        p.frame = lldp::encode(frame);
        p.neighbours.clear();
    };
    try {
        rtnl_holder = std::make_unique<nl::Rtnl>();
        nl::Rtnl& rtnl = *rtnl_holder;
        for (const auto& ifname : silent) {
            auto link = rtnl.link_by_name(ifname);
            if (!link.up()) rtnl.link_set_up(link.index);
        }
        int64_t now = mono_ns();
        for (auto& [ifname, desc] : ports) {
            Port p;
            open_port(rtnl, ifname, desc, p);
            p.next = phase == "zero" ? now : now + int64_t(std::uniform_real_distribution<double>(0, 1)(rng) * double(interval));
            // Scheduled first periodic frame (CLOCK_MONOTONIC ns): lets the harness model an
            // agent that never solicits fast start (the reference's) on the same run.
            std::printf("first %s %lld\n", ifname.c_str(), (long long)p.next);
            epoll_event ev{};
            ev.events = EPOLLIN;
            ev.data.u64 = ps.size();
            ::epoll_ctl(ep, EPOLL_CTL_ADD, p.sock->fd(), &ev);
            ps.push_back(std::move(p));
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error: %s\n", e.what());
        return 1;
    }
    std::printf("ready\n");
    std::fflush(stdout);

    pkt::ListenerStats st;
    int64_t next_port_check = mono_ns() + 100000000;
    while (!g_stop) {
        int64_t now = mono_ns(), next = INT64_MAX;
        if (now >= next_port_check) {  // a re-created port has a new ifindex: follow it
            next_port_check = now + 100000000;
            for (size_t i = 0; i < ps.size(); ++i) {
                const auto& [ifname, desc] = ports[i];
                try {
                    auto link = rtnl_holder->link_by_name(ifname);
                    if (link.index == ps[i].sock->ifindex()) continue;
                    open_port(*rtnl_holder, ifname, desc, ps[i]);
                    epoll_event ev{};
                    ev.events = EPOLLIN;
                    ev.data.u64 = i;
                    ::epoll_ctl(ep, EPOLL_CTL_ADD, ps[i].sock->fd(), &ev);
                    NLOG_V(1, "%s: port re-created, following it (ifindex %d)", ifname.c_str(), link.index);
                } catch (const std::exception&) {  // gone for now
                }
            }
        }
        bool all_done = count > 0;
        for (auto& p : ps) {
            if (count > 0 && p.periodic_sent >= count && p.fast_left == 0) continue;
            all_done = false;
            next = std::min(next, p.next);
        }
        if (all_done) break;
        int timeout = next <= now ? 0 : int(std::min<int64_t>((next - now + 999999) / 1000000, 1000));
        epoll_event evs[16];
        int n = ::epoll_wait(ep, evs, 16, timeout);
        now = mono_ns();
        for (int i = 0; i < n; ++i) {
            auto& p = ps[size_t(evs[i].data.u64)];
            for (auto& f : p.sock->drain(&st)) {
                std::string who = f.src.str();
                if (fast_start && f.ttl > 0 && p.neighbours.insert(who).second) {
                    NLOG_V(1, "%s: new neighbour %s -> fast start", p.sock->ifname().c_str(), who.c_str());
                    p.fast_left = tx_fast_init;
                    p.next = now;
                }
                if (f.ttl == 0) p.neighbours.erase(who);  // shutdown LLDPDU
            }
        }
        for (auto& p : ps) {
            if (p.next > now) continue;
            if (count > 0 && p.periodic_sent >= count && p.fast_left == 0) continue;
            try {
                p.sock->send(p.frame);
            } catch (const std::exception& e) {
                NLOG_W("send failed: %s", e.what());
            }
            if (p.fast_left > 0) {
                --p.fast_left;
                p.next = now + fast_interval;
            } else {
                ++p.periodic_sent;
                p.next = now + interval;
            }
        }
    }
    ::close(ep);
    return 0;
}
