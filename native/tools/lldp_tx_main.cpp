// `netop-lldp-tx` — synthetic ToR switch: transmits LLDPDUs on one or more interfaces.
//
// Used by the netns harness (node-ready latency bench, integration tests) to play the
// switch side of the reference's contract: a Port Description TLV carrying
// "<tag> a.b.c.d/30" per switch port (reference README.md:19-25).
//
//   netop-lldp-tx --port sw0=no-alert\ 10.200.0.2/30 --port sw1=... [--interval 1s] [--count N]
//                 [--delay 0s] [--system-name tor1] [--mac-from-port]
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <thread>

#include "netop/cli.hpp"
#include "netop/lldp.hpp"
#include "netop/log.hpp"
#include "netop/netlink.hpp"
#include "netop/packet.hpp"

using namespace netop;

static volatile sig_atomic_t g_stop = 0;
static void on_sig(int) { g_stop = 1; }

int main(int argc, char** argv) {
    std::vector<std::pair<std::string, std::string>> ports;
    int64_t interval = 1000000000LL, delay = 0;
    int count = 0;  // 0 = forever
    std::string sysname = "tor-synthetic";
    int ttl = 120, verbosity = 0;
    bool chassis_mac_is_port = true;

    cli::FlagSet fs("netop-lldp-tx");
    fs.add_func("port", true, [&](const std::string& v) {
        auto eq = v.find('=');
        if (eq == std::string::npos) throw std::invalid_argument("--port wants IFNAME=PORT_DESCRIPTION");
        ports.emplace_back(v.substr(0, eq), v.substr(eq + 1));
    }, "IFNAME=PORT_DESCRIPTION (repeatable)");
    fs.add_duration("interval", &interval, "transmit interval");
    fs.add_duration("delay", &delay, "delay before the first frame");
    fs.add_int("count", &count, "frames per port (0 = until SIGTERM)");
    fs.add_string("system-name", &sysname, "System Name TLV");
    fs.add_int("ttl", &ttl, "TTL TLV");
    fs.add_bool("mac-from-port", &chassis_mac_is_port, "chassis ID = sending port MAC");
    fs.add_int("v", &verbosity, "log verbosity");
    try {
        fs.parse(argc, argv);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error: %s\n%s", e.what(), fs.usage().c_str());
        return 2;
    }
    log::set_verbosity(verbosity);
    if (ports.empty()) {
        std::fprintf(stderr, "Error: no --port given\n");
        return 2;
    }
    signal(SIGTERM, on_sig);
    signal(SIGINT, on_sig);

    struct Tx {
        std::unique_ptr<pkt::LldpSocket> sock;
        std::vector<uint8_t> frame;
    };
    std::vector<Tx> txs;
    try {
        nl::Rtnl rtnl;
        for (auto& [ifname, desc] : ports) {
            auto link = rtnl.link_by_name(ifname);
            if (!link.up()) rtnl.link_set_up(link.index);
            auto f = lldp::make_switch_frame(link.mac, sysname, ifname, desc, uint16_t(ttl));
            txs.push_back({std::make_unique<pkt::LldpSocket>(ifname, link.index, link.mac, false), lldp::encode(f)});
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error: %s\n", e.what());
        return 1;
    }
    if (delay > 0) std::this_thread::sleep_for(std::chrono::nanoseconds(delay));
    for (int n = 0; !g_stop && (count == 0 || n < count); ++n) {
        for (auto& t : txs) {
            try {
                t.sock->send(t.frame);
                NLOG_V(2, "sent LLDP on %s", t.sock->ifname().c_str());
            } catch (const std::exception& e) {
                NLOG_W("send failed: %s", e.what());
            }
        }
        if (count != 0 && n + 1 >= count) break;
        int64_t until = mono_ns() + interval;
        while (!g_stop && mono_ns() < until) std::this_thread::sleep_for(std::chrono::milliseconds(std::min<int64_t>(50, (until - mono_ns()) / 1000000 + 1)));
    }
    return 0;
}
