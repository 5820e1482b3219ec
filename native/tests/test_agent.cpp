#include <linux/dcbnl.h>
#include <arpa/inet.h>
#include <ctime>
#include <fcntl.h>
#include <poll.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <cstddef>
#include <cstring>
#include <filesystem>
#include <set>

#include "check.hpp"
#include "fake_netops.hpp"
#include "netop/agent.hpp"
#include "netop/artifacts.hpp"
#include "netop/common.hpp"
#include "netop/topology.hpp"
#include "tmpdir.hpp"

using namespace netop;

namespace {
struct ScriptedLldp : agent::LldpSource {
    std::map<std::string, lldp::Frame> frames;
    std::map<std::string, pkt::ListenerStats> per_if;  // what stats_for reports
    std::optional<pkt::ListenerStats> stats_for(const std::string& ifname) const override {
        auto it = per_if.find(ifname);
        if (it == per_if.end()) return std::nullopt;
        return it->second;
    }
    std::vector<std::string> added;
    pkt::ListenResult result_if_unfinished = pkt::ListenResult::Deadline;
    void add(const std::string& ifname, int, const MacAddr&) override { added.push_back(ifname); }
    pkt::ListenResult run(int64_t, const std::function<bool(const std::string&, const lldp::Frame&)>& cb, int) override {
        for (auto& i : added) {
            auto it = frames.find(i);
            if (it != frames.end() && cb(i, it->second)) return pkt::ListenResult::Stopped;
        }
        return result_if_unfinished;
    }
};

struct MockDevice : nm::DeviceIf {
    std::string name;
    bool fail_set = false;
    bool* managed;
    std::string get_interface() override { return name; }
    void set_managed(bool m) override {
        if (fail_set) throw std::runtime_error("set failed");
        *managed = m;
    }
};
struct MockNm : nm::NetworkManagerIf {
    bool fail_version = false, fail_devices = false, fail_set = false;
    std::map<std::string, bool> managed{{"ens0", true}, {"ens1", true}, {"eth9", true}};
    std::map<std::string, bool>* shared = nullptr;  // outlives the mock (the agent drops it)
    std::string get_version() override {
        if (fail_version) throw std::runtime_error("no NM");
        return "1.46.0";
    }
    std::vector<std::unique_ptr<nm::DeviceIf>> get_all_devices() override {
        if (fail_devices) throw std::runtime_error("devices failed");
        std::vector<std::unique_ptr<nm::DeviceIf>> v;
        auto& table = shared ? *shared : managed;
        if (shared && shared->empty()) *shared = managed;
        for (auto& [n, m] : table) {
            auto d = std::make_unique<MockDevice>();
            d->name = n;
            d->managed = &m;
            d->fail_set = fail_set;
            v.push_back(std::move(d));
        }
        return v;
    }
};

struct Pipe {
    int fd[2];
    Pipe() {
        if (::pipe(fd) != 0) throw std::runtime_error("pipe");
    }
    ~Pipe() {
        ::close(fd[0]);
        ::close(fd[1]);
    }
    void fire() { (void)!::write(fd[1], "x", 1); }
};

lldp::Frame sw(const char* mac, const char* desc) { return lldp::make_switch_frame(*MacAddr::parse(mac), "tor", "p", desc); }

struct Fixture {
    TmpDir tmp;
    FakeNetOps ops;
    agent::Config cfg;
    Fixture() {
        ops.add_link("ens0", 10, "02:00:00:00:00:10", false);
        ops.add_link("ens1", 11, "02:00:00:00:00:11", true);
        ops.add_link("ens2", 12, "02:00:00:00:00:12", false);
        cfg.discovery.mode = topo::DiscoveryMode::None;
        cfg.interfaces = "ens0,ens1,ens2";
        cfg.configure = true;
        cfg.keep_running = true;
        cfg.wait_ns = 100000000;
        cfg.link_wait_ns = 20000000;
        cfg.carrier_wait_ns = 20000000;
        cfg.label_holddown_ns = 0;  // republished at once (the hold-down tests set their own)
        cfg.labels.dir = tmp.path + "/features.d";
        tmp.mkdir("features.d");
        cfg.rccl_net = tmp.path + "/rccl-net.json";
        cfg.status_file = tmp.path + "/status.json";
    }
    std::unique_ptr<ScriptedLldp> all_valid() {
        auto s = std::make_unique<ScriptedLldp>();
        s->frames["ens0"] = sw("02:aa:00:00:00:00", "no-alert 10.200.0.2/30");
        s->frames["ens1"] = sw("02:aa:00:00:00:01", "no-alert 10.200.0.6/30");
        s->frames["ens2"] = sw("02:aa:00:00:00:02", "no-alert 10.200.0.9/30");
        return s;
    }
    agent::NmFactory nm(std::map<std::string, bool>* out = nullptr) {
        return [out]() {
            auto m = std::make_unique<MockNm>();
            if (out) m->shared = out;
            return m;
        };
    }
};

bool has_route(FakeNetOps& o, int idx, const char* dst, const char* gw) {
    for (auto& r : o.routes)
        if (r.ifindex == idx && r.dst.masked().str() == dst && (gw ? (r.gateway && r.gateway->str() == gw) : !r.gateway))
            return true;
    return false;
}
}  // namespace

TEST(agent_l3_happy_path_and_sigterm_cleanup) {
    Fixture f;
    f.cfg.mtu = 9000;
    Pipe stop;
    stop.fire();  // SIGTERM already pending: run() returns right after publishing readiness
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    // Observe the label while "idling": write_status happens before idle, label too.
    a.run(stop.fd[0]);
    CHECK(a.ready());
    for (auto& n : a.nics()) CHECK(n.configured);
    // After SIGTERM cleanup: no label, no IPv4, originally-down links down again.
    CHECK(!path_exists(f.cfg.labels.path()));
    CHECK(f.ops.addrs.empty());
    CHECK(!(f.ops.links["ens0"].flags & IFF_UP));
    CHECK(f.ops.links["ens1"].flags & IFF_UP);
    CHECK(!(f.ops.links["ens2"].flags & IFF_UP));
    CHECK_EQ(f.ops.links["ens0"].mtu, 9000);
    auto j = read_file(f.cfg.rccl_net);
    CHECK(j && j->find("\"NIC_IP\":\"10.200.0.1\"") != std::string::npos);
    CHECK(j->find("\"NIC_IP\":\"10.200.0.10\"") != std::string::npos);
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"ready\":true") != std::string::npos && st->find("total_ready") != std::string::npos);
}

TEST(agent_l3_routes_and_label_while_running) {
    Fixture f;
    f.cfg.keep_running = false;  // configure and exit: state stays in place for inspection
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    CHECK(has_route(f.ops, 10, "10.200.0.0/30", nullptr));
    CHECK(has_route(f.ops, 10, "10.200.0.0/16", "10.200.0.2"));
    CHECK(has_route(f.ops, 11, "10.200.0.4/30", nullptr));
    CHECK(has_route(f.ops, 11, "10.200.0.0/16", "10.200.0.6"));
    CHECK(has_route(f.ops, 12, "10.200.0.8/30", nullptr));
    CHECK(has_route(f.ops, 12, "10.200.0.0/16", "10.200.0.9"));
    CHECK_EQ(f.ops.addrs.size(), size_t(3));
    CHECK(!path_exists(f.cfg.labels.path()));  // label only with --keep-running (main.go:239)
}

bool has_table_route(FakeNetOps& o, int idx, const char* dst, const char* gw, int table) {
    for (auto& r : o.routes)
        if (r.table == uint32_t(table) && r.ifindex == idx && r.dst.masked().str() == dst &&
            (gw ? (r.gateway && r.gateway->str() == gw) : !r.gateway))
            return true;
    return false;
}

TEST(agent_rail_tables_route_each_source_through_its_nic) {
    Fixture f;
    f.cfg.keep_running = false;
    f.cfg.rail_table_base = 100;
    // A previous run's rule for rail 0 (tagged with the agent's protocol) and a host rule that
    // happens to use priority 101 and table 100 (not the agent's: must survive).
    f.ops.rules.push_back(nl::RuleSpec{*Ipv4Prefix::parse("10.9.9.9/32"), 100, 100, agent::kRailProtocol});
    const nl::RuleSpec foreign{*Ipv4Prefix::parse("192.168.5.0/24"), 100, 101};
    f.ops.rules.push_back(foreign);
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    // main table unchanged (the reference's routes), plus one table per rail
    CHECK(has_route(f.ops, 10, "10.200.0.0/16", "10.200.0.2"));
    CHECK(has_table_route(f.ops, 10, "10.200.0.0/30", nullptr, 100));
    CHECK(has_table_route(f.ops, 10, "10.200.0.0/16", "10.200.0.2", 100));
    CHECK(has_table_route(f.ops, 11, "10.200.0.4/30", nullptr, 101));
    CHECK(has_table_route(f.ops, 11, "10.200.0.0/16", "10.200.0.6", 101));
    CHECK(has_table_route(f.ops, 12, "10.200.0.0/16", "10.200.0.9", 102));
    CHECK_EQ(f.ops.rules.size(), size_t(4));  // the agent's stale rule of table 100 is gone, the host's stays
    CHECK(f.ops.rules[0] == foreign);
    CHECK(f.ops.rules[1] == (nl::RuleSpec{*Ipv4Prefix::parse("10.200.0.1/32"), 100, 100, agent::kRailProtocol}));
    CHECK(f.ops.rules[3] == (nl::RuleSpec{*Ipv4Prefix::parse("10.200.0.10/32"), 102, 102, agent::kRailProtocol}));
    for (auto& r : f.ops.routes)
        if (r.table >= 100 && r.table <= 102) CHECK_EQ(int(r.protocol), int(agent::kRailProtocol));
    CHECK(a.nics()[1].configured);
}

TEST(agent_rail_indices_unique_with_unpaired_nics) {
    // Paired NICs keep their GPU index; NICs without a GPU (extra --interfaces, a GPU with no
    // NIC in reach) take the indices after the highest GPU's: no two rails share a table.
    Fixture f;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.nics_.resize(5);
    int gpu[] = {3, -1, 0, -1, 1};
    for (int i = 0; i < 5; ++i) a.nics_[size_t(i)].gpu_index = gpu[i];
    a.assign_rail_indices();
    std::vector<int> got;
    for (auto& n : a.nics_) got.push_back(n.rail_index);
    CHECK((got == std::vector<int>{3, 4, 0, 5, 1}));
}

TEST(agent_rail_routing_removed_with_the_address_it_was_installed_for) {
    // A Port Description change that yields no usable address: the old rail rule (built from the
    // old address) must still be removed -- from the record, not from n.addr.
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.rail_table_base = 100;
    Pipe stop;
    auto src = f.all_valid();
    ScriptedLldp* raw = src.get();
    agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
    bool gone = false;
    a.on_monitor_tick = [&](int tick) {
        if (tick == 1) raw->frames["ens1"] = sw("02:aa:00:00:00:01", "no-alert not-an-address");
        if (tick == 3) {
            gone = true;
            for (auto& r : f.ops.rules) gone &= r.src.addr.str() != "10.200.0.5";
            for (auto& r : f.ops.routes) gone &= r.table != 101;
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(gone);
    CHECK(f.ops.rules.empty());
}

TEST(agent_rail_tables_removed_on_sigterm) {
    Fixture f;
    f.cfg.rail_table_base = 100;
    Pipe stop;
    stop.fire();
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(stop.fd[0]);
    CHECK(a.ready());
    CHECK(f.ops.rules.empty());
    for (auto& r : f.ops.routes) CHECK(r.table < 100 || r.table > 102);
}

TEST(agent_rail_rule_failure_leaves_nic_unconfigured) {
    Fixture f;
    f.cfg.keep_running = false;
    f.cfg.rail_table_base = 100;
    f.ops.fail.insert("rule_add");
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    try {
        a.run(-1);
    } catch (...) {
    }
    for (auto& n : a.nics()) CHECK(!n.configured && !n.config_error.empty());
}

TEST(agent_reference_fixture_partial_failure) {
    // network_test.go:138-202: one valid NIC, one garbage Port Description.
    Fixture f;
    auto s = f.all_valid();
    s->frames["ens1"] = sw("02:aa:00:00:00:01", "garbage");
    agent::Agent a(f.cfg, f.ops, std::move(s), f.nm());
    bool threw = false;
    try {
        a.run(-1);
    } catch (const agent::AgentError& e) {
        threw = true;
        CHECK(std::string(e.what()).find("Not all interfaces were configured (2/3)") != std::string::npos);
    }
    CHECK(threw);
    CHECK(!path_exists(f.cfg.labels.path()));
}

TEST(agent_silent_nics_are_diagnosed_in_the_error_status_and_metrics) {
    // when --wait expires, say per NIC which driver it has and what it heard.
    Fixture f;
    f.cfg.wait_ns = 1000000;
    f.cfg.sysfs_root = f.tmp.path + "/sys/";
    // ens1 is an ionic NIC (sysfs device/driver); ens0 and ens2 have no PCI device.
    f.tmp.mkdir("sys/devices/pci0000:00/0000:00:01.0/0000:01:00.0/net/ens1");
    f.tmp.mkdir("sys/bus/pci/drivers/ionic");
    f.tmp.symlink("sys/bus/pci/drivers/ionic", "sys/devices/pci0000:00/0000:00:01.0/0000:01:00.0/driver");
    f.tmp.symlink("sys/devices/pci0000:00/0000:00:01.0/0000:01:00.0/net/ens1", "sys/class/net/ens1");
    f.tmp.symlink("sys/devices/pci0000:00/0000:00:01.0/0000:01:00.0",
                  "sys/devices/pci0000:00/0000:00:01.0/0000:01:00.0/net/ens1/device");
    auto s = f.all_valid();
    s->frames.erase("ens1");  // traffic, but no LLDPDU: a firmware agent eats them
    s->frames.erase("ens2");  // nothing at all
    f.ops.rx[11] = 100;
    f.ops.rx_step[11] = 412;
    f.ops.rx[12] = 7;
    agent::Agent a(f.cfg, f.ops, std::move(s), f.nm());
    std::string err;
    try {
        a.run(-1);
    } catch (const agent::AgentError& e) {
        err = e.what();
    }
    CHECK(err.find("Not all interfaces were configured (1/3). LLDP silent on 2 NIC(s): ") == 0);
    CHECK(err.find("ens1 (ionic: no LLDPDU in 1ms, 412 frame(s) arrived meanwhile; NIC-firmware LLDP agent suspected") !=
          std::string::npos);
    CHECK(err.find("ens2 (unknown driver: no LLDPDU in 1ms, 0 frame(s) arrived meanwhile; the link received nothing") !=
          std::string::npos);
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"driver\":\"ionic\",\"lldp_silent\":\"ionic: no LLDPDU") != std::string::npos);
    auto m = a.render_metrics();
    CHECK(m.find("netop_agent_lldp_silent{nic=\"ens1\",driver=\"ionic\"} 1") != std::string::npos);
    CHECK(m.find("netop_agent_lldp_silent{nic=\"ens2\",driver=\"\"} 1") != std::string::npos);
    CHECK(m.find("netop_agent_lldp_silent{nic=\"ens0\",driver=\"\"} 0") != std::string::npos);

    // L3 on a NIC that never got a carrier: no frame could arrive, and the reason says so.
    Fixture d;
    d.cfg.wait_ns = 1000000;
    d.ops.no_carrier = {"ens2"};
    auto sd = d.all_valid();
    sd->frames.erase("ens2");
    agent::Agent ad(d.cfg, d.ops, std::move(sd), d.nm());
    std::string derr;
    try {
        ad.run(-1);
    } catch (const agent::AgentError& e) {
        derr = e.what();
    }
    CHECK(derr.find("ens2 (unknown driver: no carrier in 1ms (check the cable, the switch port and the optic))") !=
          std::string::npos);

    // Frames that do not decode, and an i40e NIC (a known firmware-LLDP switch exists).
    Fixture g;
    g.cfg.wait_ns = 1000000;
    auto t = std::make_unique<ScriptedLldp>();
    pkt::ListenerStats bad;
    bad.malformed = 3;
    t->per_if["ens0"] = bad;
    g.ops.rx[10] = 0;
    g.ops.rx_step[10] = 5;
    agent::Agent b(g.cfg, g.ops, std::move(t), g.nm());
    err.clear();
    try {
        b.run(-1);
    } catch (const agent::AgentError& e) {
        err = e.what();
    }
    CHECK(err.find("No LLDP peers with a /30 Port Description were found. LLDP silent on 3 NIC(s): ") == 0);
    CHECK(err.find("ens0 (unknown driver: no LLDPDU in 1ms, 5 frame(s) arrived meanwhile; 3 LLDPDU(s) did not decode)") !=
          std::string::npos);
    CHECK(err.find("ens1 (unknown driver: no LLDPDU in 1ms, receive counters unavailable; NIC-firmware") != std::string::npos);

    // The counters themselves failing is only less information, never an agent failure of its own.
    Fixture h;
    h.cfg.wait_ns = 1000000;
    h.ops.fail.insert("link_stats");
    agent::Agent c(h.cfg, h.ops, std::make_unique<ScriptedLldp>(), h.nm());
    err.clear();
    try {
        c.run(-1);
    } catch (const agent::AgentError& e) {
        err = e.what();
    }
    CHECK(err.find("No LLDP peers with a /30 Port Description were found. LLDP silent on 3 NIC(s): ") == 0);
    CHECK(err.find("receive counters unavailable") != std::string::npos);
}

TEST(agent_no_peers_is_an_error_unless_compat) {
    Fixture f;
    auto s = std::make_unique<ScriptedLldp>();
    agent::Agent a(f.cfg, f.ops, std::move(s), f.nm());
    CHECK_THROWS(a.run(-1));
    Fixture g;
    g.cfg.label_without_peers = true;  // reference quirk (main.go:212,239-246)
    g.cfg.keep_running = true;
    Pipe stop;
    stop.fire();
    std::string label_seen;
    agent::Agent b(g.cfg, g.ops, std::make_unique<ScriptedLldp>(), g.nm());
    b.run(stop.fd[0]);
    CHECK(b.ready());
}

TEST(agent_l2_mode) {
    Fixture f;
    f.cfg.mode = "l2";
    f.cfg.keep_running = false;
    f.ops.addrs.push_back(nl::AddrInfo{10, AF_INET, *Ipv4::parse("192.168.1.5"), *Ipv4::parse("192.168.1.5"), 24, 0, ""});
    agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
    a.run(-1);
    CHECK(f.ops.addrs.empty());  // existing IPv4 flushed, no new ones
    CHECK(f.ops.links["ens0"].flags & IFF_UP);
    CHECK(f.ops.links["ens2"].flags & IFF_UP);
}

TEST(agent_diagnostic_run_restores_down) {
    Fixture f;
    f.cfg.configure = false;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    CHECK(f.ops.addrs.empty());
    CHECK(!(f.ops.links["ens0"].flags & IFF_UP));
    CHECK(f.ops.links["ens1"].flags & IFF_UP);
    for (auto& n : a.nics()) CHECK(n.addr);  // addresses were derived but not applied
}

TEST(agent_missing_or_no_interfaces) {
    Fixture f;
    f.cfg.interfaces = "ens0,nope";
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    bool threw = false;
    try {
        a.run(-1);
    } catch (const agent::AgentError& e) {
        threw = std::string(e.what()) == "Not all interfaces were found in the system";
    }
    CHECK(threw);
    Fixture g;
    g.cfg.interfaces = "";
    agent::Agent b(g.cfg, g.ops, g.all_valid(), g.nm());
    threw = false;
    try {
        b.run(-1);
    } catch (const agent::AgentError& e) {
        threw = std::string(e.what()) == "No interfaces found";
    }
    CHECK(threw);
    // Duplicates are de-duplicated (the reference would fail them as "not found").
    Fixture h;
    h.cfg.interfaces = "ens0,ens0, ens1 ,ens2";
    h.cfg.keep_running = false;
    agent::Agent c(h.cfg, h.ops, h.all_valid(), h.nm());
    c.run(-1);
    CHECK_EQ(c.nics().size(), size_t(3));
}

TEST(agent_sanitize) {
    agent::Config c;
    c.mtu = 100;
    c.mode = "l3";
    agent::sanitize(c);
    CHECK_EQ(c.mtu, 1500);
    CHECK_EQ(c.mode, std::string("L3"));
    c.mtu = 100000;
    agent::sanitize(c);
    CHECK_EQ(c.mtu, 9000);
    c.mode = "L4";
    CHECK_THROWS(agent::sanitize(c));
}

TEST(agent_fault_injection_nonfatal_ops) {
    for (const char* op : {"link_set_up", "link_set_mtu"}) {
        Fixture f;
        f.cfg.keep_running = false;
        f.cfg.interfaces = "ens1";  // already up: LLDP still runs
        f.ops.fail.insert(op);
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        a.run(-1);
        CHECK(a.nics()[0].configured);
    }
}

TEST(agent_fault_injection_fatal_ops) {
    for (const char* op : {"addr_list", "subscribe_links"}) {
        Fixture f;
        f.ops.fail.insert(op);
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        CHECK_THROWS(a.run(-1));
    }
    Fixture g;
    g.ops.addrs.push_back(nl::AddrInfo{10, AF_INET, *Ipv4::parse("192.168.1.5"), *Ipv4::parse("192.168.1.5"), 24, 0, ""});
    g.ops.fail.insert("addr_del");
    agent::Agent b(g.cfg, g.ops, g.all_valid(), g.nm());
    bool threw = false;
    try {
        b.run(-1);
    } catch (const agent::AgentError& e) {
        threw = std::string(e.what()).find("Failed to remove any existing IPs") == 0;
    }
    CHECK(threw);
}

TEST(agent_configure_interface_paths) {
    Fixture f;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    f.cfg.keep_running = false;
    // Build state through a diagnostic run, then drive configure_interface directly.
    agent::Config c = f.cfg;
    c.configure = false;
    agent::Agent d(c, f.ops, f.all_valid(), f.nm());
    d.run(-1);
    auto nics = d.nics();
    // Already-configured address: the /30 route must be ensured explicitly (network.go:446-452).
    f.ops.links["ens1"].flags |= IFF_UP;
    f.ops.addrs.push_back(nl::AddrInfo{11, AF_INET, *Ipv4::parse("10.200.0.5"), *Ipv4::parse("10.200.0.5"), 30, 0, ""});
    agent::Agent e(c, f.ops, f.all_valid(), f.nm());
    NicState n = nics[1];
    CHECK(e.configure_interface(n));
    CHECK(has_route(f.ops, 11, "10.200.0.4/30", nullptr));
    CHECK(has_route(f.ops, 11, "10.200.0.0/16", "10.200.0.6"));
    // Second call: EEXIST on both routes is success.
    n.configured = false;
    CHECK(e.configure_interface(n));
    // addr_add failure -> not configured
    NicState m = nics[0];
    f.ops.fail.insert("addr_add");
    CHECK(!e.configure_interface(m));
    f.ops.fail.clear();
    f.ops.fail.insert("route_append");
    CHECK(!e.configure_interface(m));
    CHECK(!m.config_error.empty());
}

TEST(agent_interrupted_during_lldp) {
    Fixture f;
    auto s = std::make_unique<ScriptedLldp>();
    s->result_if_unfinished = pkt::ListenResult::Interrupted;
    agent::Agent a(f.cfg, f.ops, std::move(s), f.nm());
    a.run(-1);
    CHECK(!a.ready());
    CHECK(!(f.ops.links["ens0"].flags & IFF_UP));
    CHECK(!path_exists(f.cfg.labels.path()));
}

TEST(agent_networkmanager_paths) {
    Fixture f;
    f.cfg.disable_nm = true;
    f.cfg.keep_running = false;
    f.cfg.nm_keyfile_dir = f.tmp.path + "/NetworkManager/conf.d";
    f.tmp.mkdir("NetworkManager");
    std::map<std::string, bool> seen;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm(&seen));
    a.run(-1);
    CHECK_EQ(seen.size(), size_t(3));
    CHECK(!seen["ens0"]);
    CHECK(!seen["ens1"]);
    CHECK(seen["eth9"]);
    auto kf = read_file(f.cfg.nm_keyfile_dir + "/99-amd-network-operator.conf");
    CHECK(kf && kf->find("unmanaged-devices+=interface-name:ens0;interface-name:ens1;interface-name:ens2") != std::string::npos);

    // NM absent (version query fails) -> silently skipped (networkmanager.go:81-86).
    MockNm nm1;
    nm1.fail_version = true;
    CHECK(nm::disable_for_interfaces(nm1, {"ens0"}).empty());
    CHECK(nm1.managed["ens0"]);
    MockNm nm2;
    nm2.fail_devices = true;
    CHECK_THROWS(nm::disable_for_interfaces(nm2, {"ens0"}));
    MockNm nm3;
    nm3.fail_set = true;
    CHECK_THROWS(nm::disable_for_interfaces(nm3, {"ens0"}));
    // Factory failure is fatal.
    Fixture g;
    g.cfg.disable_nm = true;
    agent::Agent b(g.cfg, g.ops, g.all_valid(), []() -> std::unique_ptr<nm::NetworkManagerIf> { throw std::runtime_error("no bus"); });
    CHECK_THROWS(b.run(-1));
}

TEST(agent_networkmanager_changes_undone_on_sigterm) {
    Fixture f;
    f.cfg.disable_nm = true;
    f.cfg.nm_restore = true;
    f.cfg.nm_keyfile_dir = f.tmp.path + "/NetworkManager/conf.d";
    f.tmp.mkdir("NetworkManager");
    std::map<std::string, bool> seen;
    Pipe stop;
    stop.fire();  // SIGTERM pending: run() configures, publishes, then cleans up
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm(&seen));
    a.run(stop.fd[0]);
    CHECK(a.ready());
    // The persistent keyfile is gone and NetworkManager manages the NICs again.
    CHECK(!path_exists(f.cfg.nm_keyfile_dir + "/99-amd-network-operator.conf"));
    CHECK(seen["ens0"] && seen["ens1"] && seen["eth9"]);

    // By default (--nm-restore=false) both stay: an ordinary restart (rolling update, drain,
    // reboot) must not hand the NICs back to NetworkManager (reference behaviour for Managed).
    Fixture g;
    g.cfg.disable_nm = true;
    CHECK(!g.cfg.nm_restore);
    g.cfg.nm_keyfile_dir = g.tmp.path + "/NetworkManager/conf.d";
    g.tmp.mkdir("NetworkManager");
    std::map<std::string, bool> seen2;
    Pipe stop2;
    stop2.fire();
    agent::Agent b(g.cfg, g.ops, g.all_valid(), g.nm(&seen2));
    b.run(stop2.fd[0]);
    CHECK(path_exists(g.cfg.nm_keyfile_dir + "/99-amd-network-operator.conf"));
    CHECK(!seen2["ens0"] && !seen2["ens1"] && seen2["eth9"]);
    ::unlink((g.cfg.nm_keyfile_dir + "/99-amd-network-operator.conf").c_str());

    // A file of that name the agent did not write is never deleted.
    g.tmp.write("NetworkManager/conf.d/99-amd-network-operator.conf", "[keyfile]\nunmanaged-devices=mac:aa\n");
    CHECK(!nm::remove_keyfile(g.cfg.nm_keyfile_dir));
    CHECK(path_exists(g.cfg.nm_keyfile_dir + "/99-amd-network-operator.conf"));
}

TEST(agent_networkmanager_keyfiles_of_two_agents_on_one_node_coexist) {
    // An amd-so and a host-nic agent on one node, both taking their NICs from NetworkManager:
    // each has its own keyfile, both append to the unmanaged list, and one's hand-back leaves the
    // other's NICs unmanaged.
    CHECK_EQ(nm::keyfile_name(""), std::string("99-amd-network-operator.conf"));
    CHECK_EQ(nm::keyfile_name("scale-out-readiness.txt"), std::string("99-amd-network-operator.conf"));
    CHECK_EQ(nm::keyfile_name("host-nic-readiness.txt"), std::string("99-amd-network-operator-host-nic-readiness.conf"));
    Fixture f;
    f.cfg.disable_nm = true;
    f.cfg.nm_restore = true;
    f.cfg.nm_keyfile_dir = f.tmp.path + "/NetworkManager/conf.d";
    f.tmp.mkdir("NetworkManager");
    agent::Config host = f.cfg;
    host.interfaces = "ens2";
    host.labels.file = "host-nic-readiness.txt";
    host.labels.key = "amd.feature.node.kubernetes.io/host-nic-ready";
    host.keep_running = false;
    f.cfg.interfaces = "ens0,ens1";
    {
        agent::Agent h(host, f.ops, f.all_valid(), f.nm());
        h.run(-1);
    }
    Pipe stop;
    stop.fire();
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(stop.fd[0]);  // configures, then SIGTERM with --nm-restore: removes only its own file
    CHECK(!path_exists(f.cfg.nm_keyfile_dir + "/99-amd-network-operator.conf"));
    auto kf = read_file(f.cfg.nm_keyfile_dir + "/99-amd-network-operator-host-nic-readiness.conf");
    CHECK(kf && kf->find("unmanaged-devices+=interface-name:ens2\n") != std::string::npos);
}

TEST(agent_stale_label_removed_and_networkd) {
    Fixture f;
    f.tmp.write("features.d/scale-out-readiness.txt", "stale\n");
    f.cfg.keep_running = false;
    f.cfg.networkd = f.tmp.path + "/networkd";
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    CHECK(!path_exists(f.cfg.labels.path()));
    CHECK(path_exists(f.cfg.networkd + "/ens0.network"));
    CHECK(path_exists(f.cfg.networkd + "/ens2.network"));
}

TEST(agent_monitor_link_failure_withdraws_and_restores_label) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    Pipe stop;
    auto src = f.all_valid();
    agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
    bool saw_withdrawn = false, saw_restored = false;
    a.on_monitor_tick = [&](int tick) {
        auto& l = f.ops.links["ens2"];
        if (tick == 1) {
            CHECK(path_exists(f.cfg.labels.path()));
            // the link goes administratively down: the kernel flushes its routes
            l.flags &= ~unsigned(IFF_UP);
            f.ops.routes.erase(std::remove_if(f.ops.routes.begin(), f.ops.routes.end(),
                                              [&](const nl::RouteSpec& r) { return r.ifindex == l.index; }),
                               f.ops.routes.end());
            f.ops.events.push_back({false, l});
        } else if (tick == 3) {
            saw_withdrawn = !path_exists(f.cfg.labels.path());
            // what the readiness probe prints (the kubelet puts it in the Pod's events)
            auto why = read_file(agent::reason_path(f.cfg.status_file));
            saw_withdrawn &= why && *why == "ens2: link down\n";
            l.flags |= IFF_UP;
            f.ops.events.push_back({false, l});
        } else if (tick == 5) {
            saw_restored = path_exists(f.cfg.labels.path()) && !path_exists(agent::reason_path(f.cfg.status_file));
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(saw_withdrawn);
    CHECK(saw_restored);
    CHECK_EQ(a.link_flaps(), 1);
}

TEST(agent_monitor_route_reensured_after_recovery) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.keep_running = true;
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    bool routes_back = false;
    a.on_monitor_tick = [&](int tick) {
        auto& l = f.ops.links["ens0"];
        if (tick == 1) {
            l.flags &= ~unsigned(IFF_UP);
            f.ops.routes.clear();
            f.ops.events.push_back({false, l});
        } else if (tick == 2) {
            l.flags |= IFF_UP;
            f.ops.events.push_back({false, l});
        } else if (tick == 4) {
            routes_back = has_route(f.ops, 10, "10.200.0.0/16", "10.200.0.2") && has_route(f.ops, 10, "10.200.0.0/30", nullptr);
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(routes_back);
}

TEST(agent_monitor_port_description_change_reconfigures) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    Pipe stop;
    auto src = f.all_valid();
    ScriptedLldp* raw = src.get();
    agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
    bool moved = false;
    a.on_monitor_tick = [&](int tick) {
        if (tick == 1) raw->frames["ens1"] = sw("02:aa:00:00:00:01", "no-alert 10.201.7.2/30");
        if (tick == 3) {
            bool has_new = false, has_old = false;
            for (auto& ad : f.ops.addrs) {
                if (ad.ifindex != 11) continue;
                has_new |= ad.local.str() == "10.201.7.1";
                has_old |= ad.local.str() == "10.200.0.5";
            }
            moved = has_new && !has_old && has_route(f.ops, 11, "10.201.0.0/16", "10.201.7.2");
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(moved);
    CHECK_EQ(a.reconfigurations(), 1);
    auto j = read_file(f.cfg.rccl_net);
    CHECK(j && j->find("10.201.7.1") != std::string::npos);
}

TEST(agent_monitor_rail_tables_follow_flaps_and_readdressing) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.rail_table_base = 100;
    Pipe stop;
    auto src = f.all_valid();
    ScriptedLldp* raw = src.get();
    agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
    bool back = false, moved = false;
    a.on_monitor_tick = [&](int tick) {
        auto& l = f.ops.links["ens0"];
        if (tick == 1) {  // admin down flushes every route of the device, in every table
            l.flags &= ~unsigned(IFF_UP);
            f.ops.routes.erase(std::remove_if(f.ops.routes.begin(), f.ops.routes.end(),
                                              [](const nl::RouteSpec& r) { return r.ifindex == 10; }),
                               f.ops.routes.end());
            f.ops.events.push_back({false, l});
        } else if (tick == 2) {
            l.flags |= IFF_UP;
            f.ops.events.push_back({false, l});
        } else if (tick == 4) {
            back = has_table_route(f.ops, 10, "10.200.0.0/16", "10.200.0.2", 100) &&
                   has_table_route(f.ops, 10, "10.200.0.0/30", nullptr, 100);
            raw->frames["ens1"] = sw("02:aa:00:00:00:01", "no-alert 10.201.7.2/30");
        } else if (tick == 6) {
            bool new_rule = false, old_rule = false;
            for (auto& r : f.ops.rules) {
                new_rule |= r == nl::RuleSpec{*Ipv4Prefix::parse("10.201.7.1/32"), 101, 101, agent::kRailProtocol};
                old_rule |= r.src.addr.str() == "10.200.0.5";
            }
            moved = new_rule && !old_rule && has_table_route(f.ops, 11, "10.201.0.0/16", "10.201.7.2", 101);
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(back);
    CHECK(moved);
    CHECK(f.ops.rules.empty());  // SIGTERM cleanup
}

TEST(agent_metrics_endpoint) {
    Fixture f;
    f.cfg.metrics_addr = "127.0.0.1:0";
    f.cfg.monitor_tick_ns = 1000000;
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    std::string body, ready;
    a.on_monitor_tick = [&](int tick) {
        if (tick != 1) return;
        auto get = [&](const char* path) {
            int fd = ::socket(AF_INET, SOCK_STREAM, 0);
            sockaddr_in sa{};
            sa.sin_family = AF_INET;
            sa.sin_port = htons(uint16_t(a.metrics_port()));
            sa.sin_addr.s_addr = htonl(0x7f000001);
            if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) return std::string();
            std::string req = std::string("GET ") + path + " HTTP/1.1\r\nHost: x\r\n\r\n";
            (void)!::write(fd, req.data(), req.size());
            std::string out;
            char buf[4096];
            ssize_t n;
            while ((n = ::read(fd, buf, sizeof buf)) > 0) out.append(buf, size_t(n));
            ::close(fd);
            return out;
        };
        body = get("/metrics");
        ready = get("/readyz");
        stop.fire();
    };
    a.run(stop.fd[0]);
    CHECK(body.find("HTTP/1.1 200 OK") == 0);
    CHECK(body.find("netop_agent_ready{mode=\"L3\"} 1") != std::string::npos);
    CHECK(body.find("netop_agent_nic_configured{nic=\"ens0\"") != std::string::npos);
    CHECK(body.find("netop_agent_phase_seconds{phase=\"lldp\"}") != std::string::npos);
    CHECK(ready.find("200 OK") != std::string::npos);
}

namespace {
// ethtool private-flag table per interface; "eopnotsupp" NICs have no private flags at all.
struct FakeEthtool : ethtool::Ops {
    std::map<std::string, ethtool::PrivFlags> flags;
    std::map<std::string, std::string> drivers;
    std::vector<std::pair<std::string, uint32_t>> sets;
    std::string driver(const std::string& i) override { return drivers.count(i) ? drivers[i] : ""; }
    ethtool::PrivFlags get(const std::string& i) override {
        auto it = flags.find(i);
        if (it == flags.end()) throw SysError(EOPNOTSUPP, "no private flags");
        return it->second;
    }
    void set(const std::string& i, uint32_t bits) override {
        sets.emplace_back(i, bits);
        flags[i].bits = bits;
    }
    // DCB netlink: NICs absent from `dcbx` have no DCB interface.  Setting follows mlx5_core's
    // dcbnl setdcbx: LLD_MANAGED refused, 0 = back to firmware control, else HOST required.
    std::map<std::string, uint8_t> dcbx;
    std::vector<std::pair<std::string, uint8_t>> dcbx_sets;
    std::optional<uint8_t> dcbx_get(const std::string& i) override {
        auto it = dcbx.find(i);
        if (it == dcbx.end()) return std::nullopt;
        return it->second;
    }
    bool dcbx_set(const std::string& i, uint8_t mode) override {
        dcbx_sets.emplace_back(i, mode);
        if (!dcbx.count(i)) throw SysError(EOPNOTSUPP, "DCB " + i);
        if (mode & DCB_CAP_DCBX_LLD_MANAGED) return false;
        if (mode == 0) {
            dcbx[i] = DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE;
            return true;
        }
        if (!(mode & DCB_CAP_DCBX_HOST)) return false;
        dcbx[i] = mode;
        return true;
    }
};
}  // namespace

TEST(ethtool_dcbx_handed_to_the_host_and_back) {
    // mlx5_core in firmware ("auto") DCBX mode has no private flag for its LLDP agent: the
    // driver-neutral DCBX mode says an embedded agent holds the port, and host mode takes it back.
    FakeEthtool e;
    e.drivers = {{"mlx0", "mlx5_core"}, {"mlx1", "mlx5_core"}, {"ionic0", "ionic"}};
    e.flags["mlx0"] = {{"rx_cqe_moder", "tx_cqe_moder", "rx_cqe_compress"}, 0x1};
    e.flags["mlx1"] = e.flags["mlx0"];
    e.dcbx["mlx0"] = DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE;                      // firmware
    e.dcbx["mlx1"] = DCB_CAP_DCBX_HOST | DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE;  // host already
    CHECK_EQ(ethtool::dcbx_str(0x0c), std::string("0x0c (firmware, cee, ieee)"));
    CHECK_EQ(ethtool::dcbx_str(0x06), std::string("0x06 (lld-managed, cee)"));
    CHECK(ethtool::dcbx_embedded(0x0c) && ethtool::dcbx_embedded(0x06) && !ethtool::dcbx_embedded(0x0d));
    auto rules = ethtool::builtin_rules();
    // Without the opt-in (--fw-lldp-dcbx-host) the mode is only read: the firmware keeps
    // negotiating PFC/ETS with the switch.
    auto ro = ethtool::disable_fw_lldp(e, "mlx0", rules);
    CHECK(!ro.dcbx_changed && ro.dcbx && e.dcbx_sets.empty());
    CHECK_EQ(ro.summary(), std::string("no firmware LLDP flag; DCBX 0x0c (firmware, cee, ieee)"));
    auto a = ethtool::disable_fw_lldp(e, "mlx0", rules, true, true);
    CHECK(a.dcbx_changed && !a.changed && a.error.empty());
    CHECK_EQ(int(e.dcbx["mlx0"]), 0x0d);
    CHECK_EQ(a.summary(), std::string("DCBX handed to the host (was 0x0c (firmware, cee, ieee))"));
    auto b = ethtool::disable_fw_lldp(e, "mlx1", rules, true, true);
    CHECK(!b.dcbx_changed && b.summary() == "no firmware LLDP flag; DCBX 0x0d (host, cee, ieee)");
    auto c = ethtool::disable_fw_lldp(e, "ionic0", rules, true, true);  // no private flags, no DCB interface
    CHECK(!c.dcbx && !c.dcbx_changed && c.error.empty() && c.summary() == "no firmware LLDP flag");
    // Restore: the original mode is refused by mlx5 (no HOST bit, not 0), so 0 hands it back.
    ethtool::restore(e, a);
    ethtool::restore(e, b);
    CHECK_EQ(int(e.dcbx["mlx0"]), 0x0c);
    CHECK_EQ(e.dcbx_sets.size(), size_t(3));
    CHECK(e.dcbx_sets[1] == std::make_pair(std::string("mlx0"), uint8_t(0x0c)));
    CHECK(e.dcbx_sets[2] == std::make_pair(std::string("mlx0"), uint8_t(0)));
    // A private-flag driver (ice) never gets its DCBX mode changed by the agent.
    e.drivers["ice0"] = "ice";
    e.flags["ice0"] = {{"link-down-on-close", "fw-lldp-agent"}, 0x2};
    e.dcbx["ice0"] = DCB_CAP_DCBX_LLD_MANAGED | DCB_CAP_DCBX_VER_IEEE;
    auto d = ethtool::disable_fw_lldp(e, "ice0", rules, true, true);
    CHECK(d.changed && !d.dcbx_changed && e.dcbx_sets.size() == size_t(3));
    // A driver refusing host mode is an error the status shows, not an exception.
    e.dcbx["odd0"] = DCB_CAP_DCBX_LLD_MANAGED;
    struct Refusing : FakeEthtool {
        bool dcbx_set(const std::string&, uint8_t) override { return false; }
    } r;
    r.dcbx["odd0"] = DCB_CAP_DCBX_LLD_MANAGED;
    auto f = ethtool::disable_fw_lldp(r, "odd0", rules, true, true);
    CHECK(!f.dcbx_changed && f.error.find("refused DCBX host mode 0x09 (host, ieee)") != std::string::npos);
}

TEST(agent_silent_nic_names_its_embedded_dcbx_agent) {
    // A NIC hearing traffic but no LLDPDU, whose DCBX an embedded agent holds: the diagnosis says
    // so with the mode; a host-managed one points at the switch instead.
    Fixture f;
    f.cfg.wait_ns = 1000000;
    auto s = f.all_valid();
    s->frames.erase("ens1");
    s->frames.erase("ens2");
    f.ops.rx[11] = 0;
    f.ops.rx_step[11] = 40;
    f.ops.rx[12] = 0;
    f.ops.rx_step[12] = 40;
    auto eth = std::make_unique<FakeEthtool>();
    eth->drivers = {{"ens1", "mlx5_core"}, {"ens2", "mlx5_core"}};
    eth->dcbx["ens1"] = DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE;
    eth->dcbx["ens2"] = DCB_CAP_DCBX_HOST | DCB_CAP_DCBX_VER_IEEE;
    agent::Agent a(f.cfg, f.ops, std::move(s), f.nm());
    a.set_ethtool_ops(std::move(eth));
    std::string err;
    try {
        a.run(-1);
    } catch (const agent::AgentError& e) {
        err = e.what();
    }
    CHECK(err.find("ens1 (mlx5_core: no LLDPDU in 1ms, 40 frame(s) arrived meanwhile; the NIC's embedded agent runs "
                   "DCBX and LLDP on this port (DCBX 0x0c (firmware, cee, ieee)): run with --disable-fw-lldp") !=
          std::string::npos);
    CHECK(err.find("ens2 (mlx5_core: no LLDPDU in 1ms, 40 frame(s) arrived meanwhile; DCBX is host-managed (0x09 "
                   "(host, ieee))") != std::string::npos);
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"dcbx\":\"0x0c (firmware, cee, ieee)\"") != std::string::npos);
    auto m = a.render_metrics();
    CHECK(m.find("netop_agent_dcbx_embedded{nic=\"ens1\"} 1") != std::string::npos);
    CHECK(m.find("netop_agent_dcbx_embedded{nic=\"ens2\"} 0") != std::string::npos);
    CHECK(m.find("netop_agent_dcbx_embedded{nic=\"ens0\"}") == std::string::npos);
}

TEST(ethtool_rules_parse) {
    auto r = ethtool::parse_rules(" lldp-offload=off, my-flag=1 ");
    CHECK_EQ(r.size(), size_t(4));
    CHECK_EQ(r[0].name, std::string("lldp-offload"));
    CHECK(!r[0].value && r[1].value);
    CHECK_EQ(r[2].name, std::string("disable-fw-lldp"));  // built-ins come after user rules
    CHECK_THROWS(ethtool::parse_rules("novalue"));
    CHECK_THROWS(ethtool::parse_rules("x=maybe"));
    CHECK_EQ(ethtool::parse_rules("").size(), size_t(2));
}

TEST(ethtool_disable_fw_lldp_per_driver) {
    FakeEthtool e;
    e.drivers = {{"i40e0", "i40e"}, {"ice0", "ice"}, {"mlx0", "mlx5_core"}};
    e.flags["i40e0"] = {{"MFP", "total-port-shutdown", "LinkPolling", "flow-director-atr", "veb-stats", "hw-atr-eviction",
                         "link-down-on-close", "legacy-rx", "disable-source-pruning", "disable-fw-lldp", "rs-fec"},
                        0x1};
    e.flags["ice0"] = {{"link-down-on-close", "fw-lldp-agent", "vf-true-promisc-support"}, 0x2};
    e.flags["mlx0"] = {{"rx_cqe_moder", "tx_cqe_moder", "rx_cqe_compress"}, 0x1};
    auto rules = ethtool::builtin_rules();
    auto a = ethtool::disable_fw_lldp(e, "i40e0", rules);
    CHECK(a.changed && a.error.empty());
    CHECK_EQ(e.flags["i40e0"].bits, uint32_t(0x1 | (1u << 9)));
    auto b = ethtool::disable_fw_lldp(e, "ice0", rules);
    CHECK(b.changed);
    CHECK_EQ(e.flags["ice0"].bits, uint32_t(0));
    auto c = ethtool::disable_fw_lldp(e, "mlx0", rules);
    CHECK(!c.changed && c.flag.empty() && c.error.empty());
    CHECK_EQ(c.summary(), std::string("no firmware LLDP flag"));
    auto d = ethtool::disable_fw_lldp(e, "veth0", rules);  // EOPNOTSUPP: not an error
    CHECK(!d.changed && d.error.empty());
    auto again = ethtool::disable_fw_lldp(e, "i40e0", rules);  // idempotent
    CHECK(!again.changed && again.summary() == "already disable-fw-lldp=on");
    ethtool::restore(e, a);
    ethtool::restore(e, b);
    ethtool::restore(e, c);
    CHECK_EQ(e.flags["i40e0"].bits, uint32_t(0x1));
    CHECK_EQ(e.flags["ice0"].bits, uint32_t(0x2));
    CHECK_EQ(e.sets.size(), size_t(4));
}

TEST(agent_disable_fw_lldp_and_restore_on_exit) {
    Fixture f;
    f.cfg.disable_fw_lldp = true;
    auto eth = std::make_unique<FakeEthtool>();
    eth->drivers = {{"ens0", "ice"}, {"ens1", "ice"}};
    eth->flags["ens0"] = {{"link-down-on-close", "fw-lldp-agent"}, 0x2};
    eth->flags["ens1"] = {{"link-down-on-close", "fw-lldp-agent"}, 0x0};
    FakeEthtool* raw = eth.get();
    Pipe stop;
    stop.fire();
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.set_ethtool_ops(std::move(eth));
    a.run(stop.fd[0]);
    CHECK(a.ready());
    CHECK_EQ(a.fw_lldp().size(), size_t(3));
    CHECK(a.fw_lldp()[0].changed && !a.fw_lldp()[1].changed);
    CHECK_EQ(raw->flags["ens0"].bits, uint32_t(0x2));  // restored by post_cleanups
    CHECK_EQ(raw->sets.size(), size_t(2));
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"fw_lldp\":\"set fw-lldp-agent=off\"") != std::string::npos);
    CHECK(st->find("\"fw_lldp\":\"already fw-lldp-agent=off\"") != std::string::npos);
}

TEST(agent_require_gdr) {
    Fixture f;
    f.cfg.sysfs_root = f.tmp.path + "/sys";
    f.tmp.mkdir("sys");
    f.cfg.require_gdr = "any";
    Pipe stop;
    stop.fire();
    {
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        CHECK_THROWS(a.run(stop.fd[0]));  // neither peer-memory nor ib_uverbs in the fake sysfs
    }
    f.tmp.mkdir("sys/kernel/mm/memory_peers/amdkfd");
    f.tmp.write("sys/kernel/mm/memory_peers/amdkfd/version", "1.2\n");
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(stop.fd[0]);
    CHECK(a.ready());
    CHECK_EQ(a.gdr().mode(), std::string("peermem"));
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"gpudirect_rdma\":\"peermem\"") != std::string::npos);
    CHECK(a.render_metrics().find("netop_agent_gpudirect_rdma{mode=\"peermem\"} 1") != std::string::npos);
}

namespace {
// Link events on a pollable descriptor, like the rtnetlink watcher's socket.
struct PollableNetOps : FakeNetOps {
    Pipe pipe;
    PollableNetOps() { ::fcntl(pipe.fd[0], F_SETFL, O_NONBLOCK); }
    struct Watcher : nl::LinkWatcher {
        PollableNetOps* f;
        explicit Watcher(PollableNetOps* ff) : f(ff) {}
        std::vector<nl::LinkEvent> wait(int64_t) override {
            char buf[64];
            while (::read(f->pipe.fd[0], buf, sizeof buf) > 0) {
            }
            std::vector<nl::LinkEvent> out(f->events.begin(), f->events.end());
            f->events.clear();
            return out;
        }
        int fd() const override { return f->pipe.fd[0]; }
    };
    std::unique_ptr<nl::LinkWatcher> subscribe_links() override {
        maybe_fail("subscribe_links");
        return std::make_unique<Watcher>(this);
    }
    void operational(const std::string& name) {  // linkwatch: qdisc attached, operstate UP
        auto& l = links[name];
        no_carrier.erase(name);
        l.operstate = IF_OPER_UP;
        l.flags |= IFF_LOWER_UP | IFF_RUNNING;
        events.push_back({false, l});
        pipe.fire();
    }
};

// A switch that answers a NIC only after hearing our LLDPDU on it (fast start).
struct AnsweringSwitch : agent::LldpSource {
    std::map<std::string, lldp::Frame> frames;
    std::vector<std::string> added;
    std::vector<std::pair<std::string, int>> sent;  // (ifname, TTL) of every LLDPDU we sent
    std::set<std::string> heard;
    std::function<void(int)> on_run;
    int runs = 0;
    void add(const std::string& ifname, int, const MacAddr&) override { added.push_back(ifname); }
    void announce(const std::string& ifname, const std::vector<uint8_t>& frame) override {
        auto f = lldp::decode(frame.data(), frame.size());
        sent.emplace_back(ifname, f ? int(f->ttl) : -1);
        if (f && f->ttl) heard.insert(ifname);
    }
    pkt::ListenResult run(int64_t deadline, const std::function<bool(const std::string&, const lldp::Frame&)>& cb,
                          int wait_fd) override {
        if (on_run) on_run(runs);
        ++runs;
        for (auto& i : added)
            if (heard.count(i) && cb(i, frames[i])) return pkt::ListenResult::Stopped;
        int64_t ms = std::max<int64_t>(0, (deadline - mono_ns()) / 1000000);
        pollfd p{wait_fd, POLLIN, 0};
        if (wait_fd >= 0 && ::poll(&p, 1, int(ms)) > 0) return pkt::ListenResult::Interrupted;
        if (wait_fd < 0) ::usleep(useconds_t(ms * 1000));
        return pkt::ListenResult::Deadline;
    }
};
}  // namespace

TEST(agent_announces_each_nic_when_it_becomes_operational) {
    Fixture f;
    PollableNetOps ops;
    ops.add_link("ens0", 10, "02:00:00:00:00:10", false);
    ops.add_link("ens1", 11, "02:00:00:00:00:11", false);
    ops.no_carrier = {"ens0", "ens1"};  // until linkwatch reports them operational
    f.cfg.interfaces = "ens0,ens1";
    f.cfg.lldp_announce = true;
    f.cfg.keep_running = false;
    f.cfg.wait_ns = 2000000000LL;
    auto sw_ = std::make_unique<AnsweringSwitch>();
    sw_->frames["ens0"] = sw("02:aa:00:00:00:00", "no-alert 10.200.0.2/30");
    sw_->frames["ens1"] = sw("02:aa:00:00:00:01", "no-alert 10.200.0.6/30");
    auto* s = sw_.get();
    std::vector<std::pair<std::string, int>> sent_before_up;
    s->on_run = [&](int run) {
        if (run == 0) {  // admin-up but not operational yet: nothing may have been sent
            sent_before_up = s->sent;
            ops.operational("ens0");
            ops.operational("ens1");
        }
    };
    agent::Agent a(f.cfg, ops, std::move(sw_), f.nm());
    int64_t t0 = mono_ns();
    a.run(-1);
    CHECK(sent_before_up.empty());
    // shutdown + announce per NIC, sent on its operstate-UP event, answered at once: no retry round.
    CHECK_EQ(s->sent.size(), size_t(4));
    for (auto& n : a.nics()) CHECK(n.configured);
    CHECK(mono_ns() - t0 < 250000000LL);
}

TEST(agent_retries_with_a_fresh_neighbour_when_the_answer_is_lost) {
    Fixture f;
    PollableNetOps ops;
    ops.add_link("ens0", 10, "02:00:00:00:00:10", true);
    ops.links["ens0"].operstate = IF_OPER_UP;
    f.cfg.interfaces = "ens0";
    f.cfg.lldp_announce = true;
    f.cfg.keep_running = false;
    f.cfg.wait_ns = 2000000000LL;
    auto sw_ = std::make_unique<AnsweringSwitch>();
    sw_->frames["ens0"] = sw("02:aa:00:00:00:00", "no-alert 10.200.0.2/30");
    auto* s = sw_.get();
    bool dropped = false;
    s->on_run = [&](int) {
        if (!dropped && !s->heard.empty()) {  // the switch heard us, its answer is lost
            s->heard.clear();
            dropped = true;
        }
    };
    agent::Agent a(f.cfg, ops, std::move(sw_), f.nm());
    int64_t t0 = mono_ns();
    a.run(-1);
    for (auto& n : a.nics()) CHECK(n.configured);
    // First round: shutdown + announce; the 25 ms retry: shutdown + announce again (new neighbour).
    CHECK_EQ(s->sent.size(), size_t(4));
    CHECK_EQ(s->sent[2].second, 0);
    int64_t dt = mono_ns() - t0;
    CHECK(dt >= 20000000LL && dt < 200000000LL);
}

namespace {
void write_cache(Fixture& f, int64_t age_s, const char* ens1_desc = "no-alert 10.200.0.6/30") {
    int64_t t = int64_t(::time(nullptr)) - age_s;
    artifacts::write_lldp_cache(f.cfg.lldp_cache,
                                {{"02:00:00:00:00:10", "ens0", t, "02:aa:00:00:00:00", "tor", "p", "no-alert 10.200.0.2/30"},
                                 {"02:00:00:00:00:11", "ens1", t, "02:aa:00:00:00:01", "tor", "p", ens1_desc},
                                 {"02:00:00:00:00:12", "ens2", t, "02:aa:00:00:00:02", "tor", "p", "no-alert 10.200.0.9/30"}});
}
}  // namespace

TEST(lldp_cache_roundtrip_sanitises_fields) {
    TmpDir tmp;
    std::string p = tmp.path + "/lldp-cache";
    artifacts::write_lldp_cache(p, {{"02:00:00:00:00:10", "ens0", 1700000000, "", "tor\tA", "", "no-alert\n10.0.0.2/30"}});
    auto e = artifacts::read_lldp_cache(p);
    CHECK_EQ(e.size(), size_t(1));
    CHECK_EQ(e[0].unix_s, int64_t(1700000000));
    CHECK_EQ(e[0].peer_mac, std::string(""));
    CHECK_EQ(e[0].system_name, std::string("tor A"));
    CHECK_EQ(e[0].port_description, std::string("no-alert 10.0.0.2/30"));
    write_file_atomic(p, "something else\n", 0644);  // unknown format: ignored, not misparsed
    CHECK(artifacts::read_lldp_cache(p).empty());
    CHECK(artifacts::read_lldp_cache(tmp.path + "/absent").empty());
}

TEST(agent_lldp_cache_configures_before_any_frame_then_the_switch_confirms) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
    write_cache(f, 3600);
    Pipe stop;
    auto src = std::make_unique<ScriptedLldp>();  // the switch stays silent at first
    ScriptedLldp* raw = src.get();
    agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
    bool ready_from_cache = false, confirmed = false;
    a.on_monitor_tick = [&](int tick) {
        if (tick == 0) {
            ready_from_cache = path_exists(f.cfg.labels.path()) && f.ops.addrs.size() == 3;
            auto st = read_file(f.cfg.status_file);
            ready_from_cache &= st && st->find("\"lldp_source\":\"cache\"") != std::string::npos;
            auto s2 = f.all_valid();
            raw->frames = s2->frames;
        } else if (tick == 2) {
            auto st = read_file(f.cfg.status_file);
            confirmed = st && st->find("\"lldp_source\":\"cache\"") == std::string::npos &&
                        st->find("\"lldp_source\":\"frame\"") != std::string::npos;
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(ready_from_cache);
    CHECK(confirmed);
    CHECK_EQ(a.reconfigurations(), 0);
    for (auto& e : artifacts::read_lldp_cache(f.cfg.lldp_cache))  // confirmed: timestamps refreshed
        CHECK(e.unix_s > int64_t(::time(nullptr)) - 60);
}

TEST(agent_lldp_cache_unconfirmed_withdraws_the_label_until_a_frame_arrives) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
    f.cfg.lldp_cache_confirm_ns = 30000000;  // 30 ms
    write_cache(f, 60);
    Pipe stop;
    auto src = std::make_unique<ScriptedLldp>();
    ScriptedLldp* raw = src.get();
    agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
    bool withdrawn = false, restored = false;
    int64_t t_start = mono_ns();
    int phase = 0;
    a.on_monitor_tick = [&](int) {
        if (phase == 0 && mono_ns() - t_start > 200000000) {
            withdrawn = !path_exists(f.cfg.labels.path());
            auto st = read_file(f.cfg.status_file);
            withdrawn &= st && st->find("\"cache_unconfirmed\":true") != std::string::npos;
            auto s2 = f.all_valid();
            raw->frames = s2->frames;
            phase = 1;
        } else if (phase == 1 && path_exists(f.cfg.labels.path())) {
            restored = true;
            stop.fire();
        } else if (mono_ns() - t_start > 2000000000LL) {
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(withdrawn);
    CHECK(restored);
}

TEST(agent_lldp_cache_wrong_entry_is_corrected_by_the_first_frame) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
    write_cache(f, 60, "no-alert 10.201.7.2/30");  // ens1's port was re-addressed while we were down
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.on_monitor_tick = [&](int tick) {
        if (tick == 1) stop.fire();
    };
    a.run(stop.fd[0]);
    bool has_new = false, has_old = false;
    for (auto& n : a.nics())
        if (n.ifname == "ens1") has_new = n.addr && n.addr->local.str() == "10.200.0.5";
    for (auto& ad : f.ops.addrs) has_old |= ad.local.str() == "10.201.7.1";
    CHECK(has_new);
    CHECK(!has_old);
    for (auto& e : artifacts::read_lldp_cache(f.cfg.lldp_cache))
        if (e.ifname == "ens1") CHECK_EQ(e.port_description, std::string("no-alert 10.200.0.6/30"));
    CHECK_EQ(a.reconfigurations(), 1);
}

TEST(agent_lldp_cache_ignores_old_foreign_and_unmonitored_entries) {
    for (int variant = 0; variant < 3; ++variant) {
        Fixture f;
        f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
        f.cfg.wait_ns = 20000000;
        if (variant == 0) write_cache(f, 8 * 24 * 3600);  // older than max age
        if (variant == 1) {                              // the NICs were swapped: different MACs
            write_cache(f, 60);
            auto e = artifacts::read_lldp_cache(f.cfg.lldp_cache);
            for (auto& x : e) x.nic_mac = "02:00:00:00:99:99";
            artifacts::write_lldp_cache(f.cfg.lldp_cache, e);
        }
        if (variant == 2) {  // no monitor to confirm it: the cache is not used
            write_cache(f, 60);
            f.cfg.keep_running = false;
        }
        agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
        Pipe stop;
        stop.fire();
        try {
            a.run(stop.fd[0]);
        } catch (const std::exception&) {
        }
        CHECK(f.ops.addrs.empty());
        CHECK(!a.ready());
    }
}

TEST(agent_topology_file_generated_off_the_critical_path) {
    Fixture f;
    f.cfg.keep_running = false;
    f.cfg.rccl_topo = f.tmp.path + "/rccl-topo.xml";
    f.cfg.rccl_topo_env_path = "/etc/amd/scale-out/rccl-topo.xml";
    f.cfg.rccl_env = f.tmp.path + "/rccl.env";
    f.cfg.sysfs_root = f.tmp.path + "/sys/";  // no PCI devices: a tree with no GPUs
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    auto xml = read_file(f.cfg.rccl_topo);
    CHECK(xml && xml->rfind("<system version=\"2\">", 0) == 0);
    auto env = read_file(f.cfg.rccl_env);
    CHECK(env && env->find("NCCL_TOPO_FILE=/etc/amd/scale-out/rccl-topo.xml\n") != std::string::npos);
}

TEST(agent_late_topology_worker_is_not_waited_for_and_rccl_env_names_its_file_once_it_answers) {
    // The topology worker stalls (here: its reuse key is a FIFO nobody writes yet, as a bridge
    // attribute in PCIe error recovery would): the start waits --sysfs-read-timeout for it, labels
    // the node with an rccl.env that names no NCCL_TOPO_FILE, and the monitor writes the file and
    // names it once the worker answers.
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.sysfs_read_timeout_ns = 20000000;  // 20 ms
    f.cfg.rccl_topo = f.tmp.path + "/rccl-topo.xml";
    f.cfg.rccl_env = f.tmp.path + "/rccl.env";
    f.cfg.sysfs_root = f.tmp.path + "/sys/";
    const std::string key = f.cfg.rccl_topo + ".key";
    CHECK_EQ(::mkfifo(key.c_str(), 0600), 0);
    auto release = [&] {  // the worker is blocked opening the FIFO: a writer lets it read "no match"
        int w = ::open(key.c_str(), O_WRONLY | O_NONBLOCK | O_CLOEXEC);
        if (w < 0) return false;
        (void)!::write(w, "another boot\n", 13);
        ::close(w);
        return true;
    };
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    bool labelled_without = false, released = false, named = false;
    const int64_t t0 = mono_ns();
    a.on_monitor_tick = [&](int) {
        auto env = read_file(f.cfg.rccl_env);
        if (!released) {
            labelled_without = path_exists(f.cfg.labels.path()) && env && env->find("NCCL_TOPO_FILE") == std::string::npos;
            released = release();
        } else if (env && env->find("NCCL_TOPO_FILE=" + f.cfg.rccl_topo + "\n") != std::string::npos) {
            named = true;
            stop.fire();
        }
        if (mono_ns() - t0 > 5000000000LL) stop.fire();
    };
    a.run(stop.fd[0]);
    if (!released) release();
    CHECK(labelled_without);
    CHECK(released && named);
    auto xml = read_file(f.cfg.rccl_topo);
    CHECK(xml && xml->rfind("<system version=\"2\">", 0) == 0);
}

TEST(agent_dry_run_changes_nothing) {
    Fixture f;
    f.cfg.dry_run = true;
    f.cfg.rccl_topo = f.tmp.path + "/rccl-topo.xml";
    f.cfg.sysfs_root = f.tmp.path + "/sys/";
    f.cfg.interfaces = "ens0,ens1,ens2,ens404";  // one not in this namespace: reported, not fatal
    auto before = f.ops.links;
    write_file_atomic(f.cfg.labels.path(), "stale=true\n", 0644);
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    CHECK(f.ops.addrs.empty());
    CHECK(f.ops.routes.empty());
    for (auto& [name, l] : before) CHECK_EQ(f.ops.links[name].flags, l.flags);
    CHECK(path_exists(f.cfg.labels.path()));  // not even the stale label is touched
    CHECK(path_exists(f.cfg.rccl_topo));
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"dry_run\":\"true\"") != std::string::npos);
    CHECK(st->find("\"not_in_netns\":\"ens404\"") != std::string::npos);
    CHECK(!a.ready());
}

TEST(agent_dry_run_reports_what_disable_fw_lldp_would_change) {
    Fixture f;
    f.cfg.dry_run = true;
    f.cfg.disable_fw_lldp = true;
    f.cfg.fw_lldp_dcbx_host = true;
    f.cfg.sysfs_root = f.tmp.path + "/sys/";
    auto eth = std::make_unique<FakeEthtool>();
    eth->drivers = {{"ens0", "ice"}, {"ens1", "mlx5_core"}, {"ens2", "mlx5_core"}};
    eth->flags["ens0"] = {{"link-down-on-close", "fw-lldp-agent"}, 0x2};
    eth->dcbx["ens1"] = DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE;
    eth->dcbx["ens2"] = DCB_CAP_DCBX_HOST | DCB_CAP_DCBX_VER_IEEE;
    FakeEthtool* raw = eth.get();
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.set_ethtool_ops(std::move(eth));
    a.run(-1);
    CHECK(raw->sets.empty() && raw->dcbx_sets.empty());  // nothing changed
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"fw_lldp\":\"would set fw-lldp-agent=off\"") != std::string::npos);
    CHECK(st->find("\"fw_lldp\":\"would hand DCBX to the host (now 0x0c (firmware, cee, ieee))\"") != std::string::npos);
    CHECK(st->find("\"fw_lldp\":\"no firmware LLDP flag; DCBX 0x09 (host, ieee)\"") != std::string::npos);
}

TEST(agent_dry_run_writes_intra_node_rccl_env) {
    Fixture f;
    f.cfg.dry_run = true;
    f.cfg.rccl_topo = f.tmp.path + "/rccl-topo.xml";
    f.cfg.rccl_env = f.tmp.path + "/rccl.env";
    f.cfg.rccl_env_extra = "NCCL_MIN_NCHANNELS=64";
    f.cfg.socket_ifname = "auto";
    f.cfg.sysfs_root = f.tmp.path + "/sys/";
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    auto env = read_file(f.cfg.rccl_env);
    CHECK(env && env->find("NCCL_TOPO_FILE=" + f.cfg.rccl_topo + "\n") != std::string::npos);
    CHECK(env->find("NCCL_MIN_NCHANNELS=64\n") != std::string::npos);
    // nothing configured: no HCA, GID or socket interface a job could not use yet
    CHECK(env->find("NCCL_IB_HCA") == std::string::npos);
    CHECK(env->find("NCCL_SOCKET_IFNAME") == std::string::npos);
    CHECK(env->find("NCCL_IB_GID_INDEX") == std::string::npos);
    CHECK(f.ops.addrs.empty());
}

TEST(agent_topology_file_reused_within_a_boot) {
    Fixture f;
    f.cfg.keep_running = false;
    f.cfg.rccl_topo = f.tmp.path + "/rccl-topo.xml";
    f.cfg.rccl_env = f.tmp.path + "/rccl.env";
    f.cfg.sysfs_root = f.tmp.path + "/sys/";
    {
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        a.run(-1);
    }
    auto key = read_file(f.cfg.rccl_topo + ".key");
    CHECK(key && key->find("boot ") != std::string::npos);
    // A restart in the same boot with the same devices keeps the file it finds.
    write_file_atomic(f.cfg.rccl_topo, "<system version=\"2\">\n<!-- kept -->\n</system>\n", 0644);
    {
        FakeNetOps ops2;
        ops2.add_link("ens0", 10, "02:00:00:00:00:10", false);
        ops2.add_link("ens1", 11, "02:00:00:00:00:11", true);
        ops2.add_link("ens2", 12, "02:00:00:00:00:12", false);
        agent::Agent a(f.cfg, ops2, f.all_valid(), f.nm());
        a.run(-1);
    }
    CHECK(read_file(f.cfg.rccl_topo)->find("kept") != std::string::npos);
    auto env = read_file(f.cfg.rccl_env);
    CHECK(env && env->find("NCCL_TOPO_FILE=") != std::string::npos);
    // Another boot (or other devices): regenerated.
    write_file_atomic(f.cfg.rccl_topo + ".key", "netop-rccl-topo v2\nboot another\n", 0644);
    {
        FakeNetOps ops3;
        ops3.add_link("ens0", 10, "02:00:00:00:00:10", false);
        ops3.add_link("ens1", 11, "02:00:00:00:00:11", true);
        ops3.add_link("ens2", 12, "02:00:00:00:00:12", false);
        agent::Agent a(f.cfg, ops3, f.all_valid(), f.nm());
        a.run(-1);
    }
    CHECK(read_file(f.cfg.rccl_topo)->find("kept") == std::string::npos);
    CHECK(*read_file(f.cfg.rccl_topo + ".key") == *key);
}

TEST(agent_monitor_exits_when_a_nic_is_removed) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.rail_table_base = 100;  // per-rail rules: the removed NIC's must not outlive it
    bool had_rules = false;
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    bool labelled_before = false;
    a.on_monitor_tick = [&](int tick) {
        if (tick == 1) {
            labelled_before = path_exists(f.cfg.labels.path());
            had_rules = f.ops.rules.size() == 3;
            auto l = f.ops.links["ens2"];
            f.ops.links.erase("ens2");  // driver reload: the netdev is gone (it returns as a new ifindex)
            f.ops.addrs.erase(std::remove_if(f.ops.addrs.begin(), f.ops.addrs.end(),
                                             [&](const nl::AddrInfo& x) { return x.ifindex == l.index; }),
                              f.ops.addrs.end());
            f.ops.events.push_back({true, l});
        } else if (tick > 20) {
            stop.fire();  // not reached: the agent leaves by itself
        }
    };
    bool threw = false;
    try {
        a.run(stop.fd[0]);
    } catch (const agent::AgentError& e) {
        threw = std::string(e.what()).find("ens2") != std::string::npos;
    }
    CHECK(labelled_before);
    CHECK(threw);
    CHECK(!path_exists(f.cfg.labels.path()));
    CHECK(f.ops.addrs.empty());  // the other NICs were cleaned up too
    CHECK(had_rules);
    CHECK(f.ops.rules.empty());  // the removed NIC's rail rule included
    CHECK(!a.ready());
}

// --- --verify-peers -------------------------------------------------------------------------
TEST(arp_request_encoding_and_reply_parsing) {
    auto req = arp::encode_request(*MacAddr::parse("02:00:00:00:00:10"), *Ipv4::parse("10.200.0.1"), *Ipv4::parse("10.200.0.2"));
    CHECK_EQ(req.size(), arp::kPayloadLen);
    const uint8_t head[8] = {0, 1, 8, 0, 6, 4, 0, 1};  // Ethernet, IPv4, 6, 4, who-has
    CHECK(std::equal(head, head + 8, req.begin()));
    CHECK_EQ(MacAddr::from_bytes(&req[8]).str(), std::string("02:00:00:00:00:10"));
    CHECK_EQ(Ipv4::from_net(&req[14]).str(), std::string("10.200.0.1"));
    CHECK(MacAddr::from_bytes(&req[18]).is_zero());
    CHECK_EQ(Ipv4::from_net(&req[24]).str(), std::string("10.200.0.2"));
    CHECK(!arp::parse_reply(req.data(), req.size()));  // a request is not a reply
    // the peer's answer: op 2, sender = the peer
    std::vector<uint8_t> rep(req);
    rep[7] = 2;
    const uint8_t peer_mac[6] = {0x02, 0xaa, 0, 0, 0, 0};
    std::copy(peer_mac, peer_mac + 6, rep.begin() + 8);
    Ipv4::parse("10.200.0.2")->to_net(&rep[14]);
    std::copy(req.begin() + 8, req.begin() + 14, rep.begin() + 18);
    Ipv4::parse("10.200.0.1")->to_net(&rep[24]);
    auto r = arp::parse_reply(rep.data(), rep.size());
    CHECK(r && r->sender_ip.str() == "10.200.0.2" && r->target_ip.str() == "10.200.0.1");
    CHECK_EQ(r->sender_mac.str(), std::string("02:aa:00:00:00:00"));
    CHECK(!arp::parse_reply(rep.data(), rep.size() - 1));  // truncated
    rep[1] = 6;                                              // IEEE 802 hardware type
    CHECK(!arp::parse_reply(rep.data(), rep.size()));
}

namespace {
// A switch whose ports answer ARP except those in `silent`; records what was asked.
struct FakeArpSwitch {
    std::set<std::string> silent;
    std::set<std::string> proxy;  // ports answering from another MAC than their LLDP one
    std::vector<std::pair<std::string, std::string>> asked;  // (ifname, peer)
    std::vector<int64_t> timeouts;                           // per probe_all call
    bool operator()(std::vector<arp::Probe>& ps, int64_t timeout_ns, int64_t, int) {
        timeouts.push_back(timeout_ns);
        for (auto& p : ps) {
            asked.push_back({p.ifname, p.peer.str()});
            p.requests = 3;
            if (silent.count(p.ifname)) continue;
            p.answered = true;
            p.rtt_ns = 120000;
            p.verify_ns = 220000;
            // the switch port's own MAC (Fixture: 02:aa:00:00:00:0k for ensk), or a proxy's
            p.peer_mac = *MacAddr::parse(proxy.count(p.ifname) ? "02:aa:00:00:00:99"
                                                               : "02:aa:00:00:00:0" + p.ifname.substr(3));
        }
        return true;
    }
};
}  // namespace

TEST(agent_verify_peers_all_answer) {
    Fixture f;
    f.cfg.keep_running = true;
    f.cfg.verify_peers_ns = 500000000;
    Pipe stop;
    stop.fire();
    FakeArpSwitch swi;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.arp_probe = [&](std::vector<arp::Probe>& ps, int64_t t, int64_t r, int s) { return swi(ps, t, r, s); };
    a.run(stop.fd[0]);
    CHECK(a.ready());
    CHECK_EQ(swi.asked.size(), size_t(3));
    std::set<std::string> peers;
    for (auto& [i, p] : swi.asked) peers.insert(i + "=" + p);
    CHECK(peers == (std::set<std::string>{"ens0=10.200.0.2", "ens1=10.200.0.6", "ens2=10.200.0.9"}));
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"peer_verified\":true") != std::string::npos && st->find("verify_peers") != std::string::npos);
    const std::string m = a.render_metrics();
    CHECK(m.find("netop_agent_peer_verified{nic=\"ens1\"} 1") != std::string::npos);
    CHECK(m.find("netop_agent_peer_arp_rtt_seconds{nic=\"ens2\"} 0.000120000") != std::string::npos);
    CHECK(m.find("netop_agent_peer_verify_seconds{nic=\"ens2\"} 0.000220000") != std::string::npos);
    CHECK(m.find("netop_agent_peer_mac_mismatch{nic=\"ens0\"} 0") != std::string::npos);
    CHECK(st->find("\"peer_verify_ms\":0.22") != std::string::npos && st->find("peer_mac_mismatch") == std::string::npos);
}

TEST(agent_verify_peers_flags_a_proxy_arp_answer) {
    // The ARP answer comes from another MAC than the LLDP peer's: flagged, not fatal.
    Fixture f;
    f.cfg.keep_running = true;
    f.cfg.verify_peers_ns = 500000000;
    Pipe stop;
    stop.fire();
    FakeArpSwitch swi;
    swi.proxy = {"ens1"};
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.arp_probe = [&](std::vector<arp::Probe>& ps, int64_t t, int64_t r, int s) { return swi(ps, t, r, s); };
    a.run(stop.fd[0]);
    CHECK(a.ready());
    const std::string m = a.render_metrics();
    CHECK(m.find("netop_agent_peer_mac_mismatch{nic=\"ens1\"} 1") != std::string::npos);
    CHECK(m.find("netop_agent_peer_mac_mismatch{nic=\"ens2\"} 0") != std::string::npos);
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"peer_arp_mac\":\"02:aa:00:00:00:99\",\"peer_mac_mismatch\":true") != std::string::npos);
}

TEST(arp_reply_must_answer_our_own_address) {
    arp::Probe p;
    p.local = *Ipv4::parse("10.200.0.1");
    p.peer = *Ipv4::parse("10.200.0.2");
    arp::Reply r;
    r.sender_mac = *MacAddr::parse("02:aa:00:00:00:00");
    r.sender_ip = p.peer;
    r.target_ip = p.local;
    CHECK(arp::answers(p, r));
    r.target_ip = *Ipv4::parse("10.200.0.5");  // aimed at another local address (another NIC)
    CHECK(!arp::answers(p, r));
    r.target_ip = p.peer;  // gratuitous: target = sender
    CHECK(!arp::answers(p, r));
    r.target_ip = p.local;
    r.sender_ip = *Ipv4::parse("10.200.0.6");  // someone else's peer
    CHECK(!arp::answers(p, r));
    // RTT vs time to verify: requests at t=1000 (first) and t=5000 (last), answer at t=5300.
    r.sender_ip = p.peer;
    arp::record_answer(p, r, 5300, 1000, 5000);
    CHECK(p.answered && p.rtt_ns == 300 && p.verify_ns == 4300);
    CHECK_EQ(p.peer_mac.str(), std::string("02:aa:00:00:00:00"));
}

TEST(agent_verify_peers_silent_peer_blocks_readiness) {
    Fixture f;
    f.cfg.keep_running = true;
    f.cfg.verify_peers_ns = 500000000;
    FakeArpSwitch swi;
    swi.silent = {"ens2"};
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.arp_probe = [&](std::vector<arp::Probe>& ps, int64_t t, int64_t r, int s) { return swi(ps, t, r, s); };
    bool threw = false;
    try {
        a.run(-1);
    } catch (const agent::AgentError& e) {
        threw = std::string(e.what()).find("1 of 3 switch-side peers did not answer ARP (ens2") != std::string::npos;
    }
    CHECK(threw);
    CHECK(!a.ready());
    CHECK(!path_exists(f.cfg.labels.path()));
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("\"peer_error\":\"peer 10.200.0.9 did not answer ARP") != std::string::npos);
    const std::string m = a.render_metrics();
    CHECK(m.find("netop_agent_peer_verified{nic=\"ens2\"} 0") != std::string::npos);
    CHECK(m.find("netop_agent_peer_arp_rtt_seconds{nic=\"ens2\"}") == std::string::npos);
}

TEST(agent_verify_peers_off_by_default_asks_nothing) {
    Fixture f;
    f.cfg.keep_running = false;
    FakeArpSwitch swi;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.arp_probe = [&](std::vector<arp::Probe>& ps, int64_t t, int64_t r, int s) { return swi(ps, t, r, s); };
    a.run(-1);
    CHECK(swi.asked.empty());
}

TEST(agent_monitor_reverifies_a_recovered_nic_before_relabelling) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.verify_peers_ns = 500000000;
    Pipe stop;
    FakeArpSwitch swi;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.arp_probe = [&](std::vector<arp::Probe>& ps, int64_t t, int64_t r, int s) { return swi(ps, t, r, s); };
    bool withdrawn = false, held_back = false, restored = false;
    size_t asked_before = 0;
    int64_t t_fixed = 0;
    a.on_monitor_tick = [&](int tick) {
        auto& l = f.ops.links["ens2"];
        if (tick == 1) {
            CHECK(path_exists(f.cfg.labels.path()));
            l.flags &= ~unsigned(IFF_UP);
            f.ops.events.push_back({false, l});
        } else if (tick == 3) {
            withdrawn = !path_exists(f.cfg.labels.path());
            swi.silent = {"ens2"};  // the port comes back without its address
            asked_before = swi.asked.size();
            l.flags |= IFF_UP;
            f.ops.events.push_back({false, l});
        } else if (tick == 6) {
            held_back = !path_exists(f.cfg.labels.path()) && swi.asked.size() > asked_before;
            swi.silent.clear();
            t_fixed = mono_ns();
        } else if (tick > 6 && path_exists(f.cfg.labels.path())) {
            restored = true;  // asked again a second after the failure; answered
            stop.fire();
        } else if (tick > 6 && mono_ns() - t_fixed > 3000000000LL) {
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(withdrawn);
    CHECK(held_back);
    CHECK(restored);
}

TEST(agent_monitor_reprobe_never_holds_the_loop_for_the_startup_timeout) {
    // Start-up waits the whole --verify-peers for a port to answer; in monitor mode a silent
    // peer is asked in short rounds so link and LLDP events on the other NICs are not delayed.
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.verify_peers_ns = 2000000000;
    Pipe stop;
    FakeArpSwitch swi;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.arp_probe = [&](std::vector<arp::Probe>& ps, int64_t t, int64_t r, int s) { return swi(ps, t, r, s); };
    a.on_monitor_tick = [&](int tick) {
        auto& l = f.ops.links["ens1"];
        if (tick == 1) {
            swi.silent = {"ens1"};
            l.flags &= ~unsigned(IFF_UP);
            f.ops.events.push_back({false, l});
        } else if (tick == 2) {
            l.flags |= IFF_UP;
            f.ops.events.push_back({false, l});
        } else if (tick > 2 && swi.timeouts.size() >= 2) {
            stop.fire();
        } else if (tick > 5000) {
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(swi.timeouts.size() >= 2);
    CHECK_EQ(swi.timeouts.front(), int64_t(2000000000));  // start-up: the configured timeout
    for (size_t i = 1; i < swi.timeouts.size(); ++i) CHECK(swi.timeouts[i] <= 250000000);
}

TEST(agent_keep_config_leaves_the_data_plane_and_the_next_agent_adopts_it) {
    // Rolling update with --keep-config: the first agent exits withdrawing only its label; the
    // second finds the addresses its LLDP cache names and keeps them (no addr_del, no addr_add),
    // so QPs bound to them never see their source address disappear.
    Fixture f;
    f.cfg.keep_config = true;
    f.cfg.rail_table_base = 100;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
    {
        Pipe stop;
        stop.fire();
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        a.run(stop.fd[0]);
        CHECK(a.ready());
    }
    CHECK(!path_exists(f.cfg.labels.path()));
    CHECK_EQ(f.ops.addrs.size(), size_t(3));
    CHECK_EQ(f.ops.rules.size(), size_t(3));
    CHECK(has_table_route(f.ops, 11, "10.200.0.0/16", "10.200.0.6", 101));
    CHECK(f.ops.links["ens0"].flags & IFF_UP);  // not put down again
    CHECK_EQ(artifacts::read_lldp_cache(f.cfg.lldp_cache).size(), size_t(3));
    // A foreign address on ens2 (not the cached /30) is still flushed.
    f.ops.addrs.push_back(nl::AddrInfo{12, AF_INET, *Ipv4::parse("192.168.77.1"), *Ipv4::parse("192.168.77.1"), 24, 0, ""});
    f.ops.calls.clear();
    {
        Pipe stop;
        auto src = std::make_unique<ScriptedLldp>();  // the switch is silent while we restart
        ScriptedLldp* raw = src.get();
        agent::Agent b(f.cfg, f.ops, std::move(src), f.nm());
        bool ready_before_frame = false;
        b.on_monitor_tick = [&](int tick) {
            if (tick == 0) {
                ready_before_frame = path_exists(f.cfg.labels.path());
                raw->frames = f.all_valid()->frames;
            }
            if (tick == 2) stop.fire();
        };
        b.run(stop.fd[0]);
        CHECK(ready_before_frame);
    }
    CHECK_EQ(f.ops.calls["addr_del"], 1);  // the foreign 192.168.77.1/24 only
    CHECK_EQ(f.ops.calls["addr_add"], 0);
    CHECK_EQ(f.ops.addrs.size(), size_t(3));
    for (auto& a : f.ops.addrs) CHECK(a.local.str() != "192.168.77.1");
    CHECK_EQ(f.ops.rules.size(), size_t(3));
}

TEST(agent_keep_config_restarts_and_readdressing_keep_every_nic_on_its_switch_ports_address) {
    // Property (L3, --keep-config, LLDP cache, rail tables): under any sequence of switch-port
    // re-addressing and agent restarts (a rolling update; half of them with the switch silent at
    // first, so the new agent starts from its cache), once an agent has caught up every NIC holds
    // exactly the /30 its switch port describes now, one rail rule each, and the node is labelled.
    // Three seeds, 30 checked steps each.
    for (uint64_t seed : {0x5EED0001ull, 0x5EED0002ull, 0x5EED0003ull}) {
        Fixture f;
        f.cfg.keep_config = true;
        f.cfg.rail_table_base = 100;
        f.cfg.monitor_tick_ns = 1000000;
        f.cfg.lldp_tx_interval_ns = 3600LL * 1000000000LL;
        f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
        const std::vector<std::string> nics = {"ens0", "ens1", "ens2"};
        const std::map<std::string, int> idx = {{"ens0", 10}, {"ens1", 11}, {"ens2", 12}};
        std::map<std::string, int> host = {{"ens0", 1}, {"ens1", 1}, {"ens2", 1}};
        auto frame = [&](const std::string& n) {
            const int k = int(n.back() - '0');
            return sw(strfmt("02:aa:00:00:00:0%d", k).c_str(), strfmt("no-alert 10.20%d.0.%d/30", k, 4 * host.at(n) + 2).c_str());
        };
        uint64_t rng = seed;
        auto next = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        int steps = 0, mismatches = 0, restarts = 0, readdressed = 0;
        std::string first_bad;
        for (int run = 0; steps < 30 && run < 40; ++run) {
            auto src = std::make_unique<ScriptedLldp>();
            ScriptedLldp* raw = src.get();
            const bool silent = run > 0 && next() % 2;  // the new agent starts from its cache
            if (!silent)
                for (const auto& n : nics) raw->frames[n] = frame(n);
            Pipe stop;
            agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
            int64_t t_step = mono_ns();
            a.on_monitor_tick = [&](int tick) {
                if (silent && tick == 3)
                    for (const auto& n : nics) raw->frames[n] = frame(n);  // the switch speaks again
                if (mono_ns() - t_step < 20000000LL) return;
                std::string bad;
                for (const auto& n : nics) {
                    const int k = int(n.back() - '0');
                    const std::string expect = strfmt("10.20%d.0.%d/30", k, 4 * host.at(n) + 1);
                    std::vector<std::string> have;
                    for (const auto& x : f.ops.addrs)
                        if (x.ifindex == idx.at(n)) have.push_back(x.prefix().str());
                    if (have != std::vector<std::string>{expect}) bad += " " + n + " holds " + join(have, ",") + " not " + expect;
                }
                if (f.ops.rules.size() != nics.size()) bad += strfmt(" %zu rail rules", f.ops.rules.size());
                if (!path_exists(f.cfg.labels.path())) bad += " no label";
                if (!bad.empty() && mono_ns() - t_step < 2000000000LL) return;  // a loaded machine: up to 2 s more
                if (!bad.empty()) {
                    if (!mismatches) first_bad = strfmt("step %d (run %d%s):", steps, run, silent ? ", cache start" : "") + bad;
                    ++mismatches;
                }
                if (++steps >= 30 || next() % 3 == 0) {  // a rolling update: this agent goes, the next comes
                    ++restarts;
                    stop.fire();
                    return;
                }
                const std::string& n = nics[next() % nics.size()];
                host[n] = 1 + int(next() % 8);
                raw->frames[n] = frame(n);
                ++readdressed;
                t_step = mono_ns();
            };
            a.run(stop.fd[0]);
        }
        if (mismatches) fprintf(stderr, "seed %llx, %s\n", (unsigned long long)seed, first_bad.c_str());
        CHECK_EQ(mismatches, 0);
        CHECK_EQ(steps, 30);
        CHECK(restarts > 3 && readdressed > 3);
    }
}

TEST(agent_l2_keep_config_rolling_restarts_under_random_cable_pulls_never_take_a_link_down) {
    // Property (L2, --keep-config, the monitor): under random cable pulls and re-plugs interleaved
    // with agent restarts (a rolling update), no agent ever sets a scale-out link down -- jobs keep
    // their links through the roll -- and once an agent has caught up the label is published
    // exactly when every NIC has carrier.  Three seeds, 60 checked steps each.
    for (uint64_t seed : {0x4C32000000000001ull, 0x4C32000000000002ull, 0x4C32000000000003ull}) {
        Fixture f;
        f.cfg.mode = "L2";
        f.cfg.keep_config = true;
        f.cfg.monitor_tick_ns = 1000000;
        f.cfg.carrier_wait_ns = 20000000;  // a restart with a pulled cable goes on to the monitor
        const std::vector<std::string> nics = {"ens0", "ens1", "ens2"};
        std::map<std::string, bool> carrier = {{"ens0", true}, {"ens1", true}, {"ens2", true}};
        uint64_t rng = seed;
        auto next = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        int steps = 0, mismatches = 0, restarts = 0, pulls = 0, labelled_states = 0;
        std::string first_bad;
        for (int run = 0; steps < 60 && run < 80; ++run) {
            Pipe stop;
            agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
            int64_t t_step = mono_ns();
            a.on_monitor_tick = [&](int) {
                if (mono_ns() - t_step < 10000000LL) return;
                const bool want = std::all_of(nics.begin(), nics.end(), [&](const std::string& n) { return carrier[n]; });
                const bool label = path_exists(f.cfg.labels.path());
                std::string bad;
                if (label != want) bad += strfmt(" label %d, want %d", label, want);
                for (const auto& n : nics)
                    if (!(f.ops.links[n].flags & IFF_UP)) bad += " " + n + " admin-down";
                if (f.ops.calls["link_set_down"]) bad += " a link was set down";
                if (!bad.empty() && mono_ns() - t_step < 2000000000LL) return;  // a loaded machine: up to 2 s more
                if (!bad.empty()) {
                    if (!mismatches) first_bad = strfmt("step %d (run %d):", steps, run) + bad;
                    ++mismatches;
                }
                labelled_states += want;
                if (++steps >= 60 || next() % 4 == 0) {  // this agent goes, the next comes
                    ++restarts;
                    stop.fire();
                    return;
                }
                const std::string& n = nics[next() % nics.size()];
                carrier[n] = !carrier[n];
                f.ops.set_carrier(n, carrier[n]);
                ++pulls;
                t_step = mono_ns();
            };
            a.run(stop.fd[0]);
        }
        if (mismatches) fprintf(stderr, "seed %llx, %s\n", (unsigned long long)seed, first_bad.c_str());
        CHECK_EQ(mismatches, 0);
        CHECK_EQ(steps, 60);
        CHECK(restarts > 5 && pulls > 20);
        CHECK(labelled_states > 0 && labelled_states < steps);  // both states visited
        CHECK_EQ(f.ops.calls["link_set_down"], 0);
    }
}

TEST(agent_keep_config_does_not_adopt_a_stale_or_foreign_cache_entry) {
    Fixture f;
    f.cfg.keep_config = true;
    f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
    f.cfg.keep_running = false;
    write_cache(f, 3600);
    auto e = artifacts::read_lldp_cache(f.cfg.lldp_cache);
    e[1].nic_mac = "02:00:00:00:00:99";  // ens1 is another card now
    e[2].unix_s -= 30LL * 24 * 3600;      // ens2's entry is too old
    artifacts::write_lldp_cache(f.cfg.lldp_cache, e);
    f.ops.addrs.push_back(nl::AddrInfo{10, AF_INET, *Ipv4::parse("10.200.0.1"), *Ipv4::parse("10.200.0.1"), 30, 0, ""});
    f.ops.addrs.push_back(nl::AddrInfo{11, AF_INET, *Ipv4::parse("10.200.0.5"), *Ipv4::parse("10.200.0.5"), 30, 0, ""});
    f.ops.addrs.push_back(nl::AddrInfo{12, AF_INET, *Ipv4::parse("10.200.0.10"), *Ipv4::parse("10.200.0.10"), 30, 0, ""});
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    CHECK_EQ(f.ops.calls["addr_del"], 2);  // ens1 and ens2 re-learn their address from LLDP
    CHECK_EQ(f.ops.addrs.size(), size_t(3));
}

TEST(agent_cleanup_mode_removes_what_kept_agents_left) {
    Fixture f;
    f.cfg.keep_config = true;
    f.cfg.rail_table_base = 100;
    f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
    f.cfg.rccl_env = f.tmp.path + "/rccl.env";
    {
        Pipe stop;
        stop.fire();
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        a.run(stop.fd[0]);
        CHECK(a.ready());
    }
    // A host rule and route the agent never made survive the cleanup.
    const nl::RuleSpec foreign{*Ipv4Prefix::parse("192.168.5.0/24"), 100, 101};
    f.ops.rules.push_back(foreign);
    nl::RouteSpec host;
    host.ifindex = 11;
    host.dst = *Ipv4Prefix::parse("172.16.0.0/12");
    host.table = 101;
    f.ops.routes.push_back(host);
    CHECK(path_exists(f.cfg.rccl_env) && path_exists(f.cfg.rccl_net) && path_exists(f.cfg.lldp_cache));
    write_file_atomic(f.cfg.labels.path(), "stale=true\n");
    agent::Config c = f.cfg;
    c.cleanup = true;
    c.keep_config = false;
    // NetworkManager: the agents left the NICs unmanaged (keyfile + Managed=false); the
    // policy-deletion cleanup (--nm-restore) hands them back.
    c.disable_nm = true;
    c.nm_restore = true;
    c.nm_keyfile_dir = f.tmp.path + "/NetworkManager/conf.d";
    f.tmp.mkdir("NetworkManager");
    CHECK(!nm::write_keyfile(c.nm_keyfile_dir, {"ens0", "ens1", "ens2"}).empty());
    std::map<std::string, bool> managed{{"ens0", false}, {"ens1", false}, {"eth9", true}};  // what NM knows
    agent::Agent k(c, f.ops, std::make_unique<ScriptedLldp>(), f.nm(&managed));
    k.run(-1);
    CHECK(!path_exists(c.nm_keyfile_dir + "/99-amd-network-operator.conf"));
    CHECK(managed["ens0"] && managed["ens1"] && managed["eth9"]);
    CHECK(f.ops.addrs.empty());
    CHECK_EQ(f.ops.rules.size(), size_t(1));
    CHECK(f.ops.rules[0] == foreign);
    for (auto& r : f.ops.routes) CHECK(r.protocol != agent::kRailProtocol);
    CHECK(std::any_of(f.ops.routes.begin(), f.ops.routes.end(), [](const nl::RouteSpec& r) { return r.table == 101; }));
    CHECK(!path_exists(f.cfg.labels.path()));
    CHECK(!path_exists(f.cfg.rccl_env) && !path_exists(f.cfg.rccl_net) && !path_exists(f.cfg.lldp_cache));
    CHECK_EQ(k.ready(), false);
    auto st = read_file(f.cfg.status_file);
    CHECK(st && st->find("cleanup") != std::string::npos);
}

TEST(ethtool_state_round_trip) {
    ethtool::FwLldpResult a, b, c;
    a.ifname = "ens0";
    a.changed = true;
    a.original_bits = 0x2;
    b.ifname = "mlx0";
    b.dcbx = uint8_t(0x0c);
    b.dcbx_changed = true;
    c.ifname = "ens9";  // nothing changed: not recorded
    auto text = ethtool::encode_state({a, b, c});
    CHECK_EQ(text, std::string("ens0 priv 0x2\nmlx0 dcbx 0x0c\n"));
    auto back = ethtool::decode_state(text + "garbage\nens1 priv zz\nens2 dcbx 0x1ff\n\n");
    CHECK_EQ(back.size(), size_t(2));
    CHECK(back[0].ifname == "ens0" && back[0].changed && back[0].original_bits == 0x2 && !back[0].dcbx_changed);
    CHECK(back[1].ifname == "mlx0" && back[1].dcbx_changed && *back[1].dcbx == 0x0c && !back[1].changed);
    // Names no interface can have (found by the fuzzer: a NUL inside one did not survive re-encoding).
    CHECK(ethtool::decode_state(std::string("e\0s0 priv 0x1\na/b priv 0x1\n.. priv 0x1\nabcdefghijklmnop priv 0x1\n", 65))
              .empty());
}

TEST(agent_failed_start_keeps_the_firmware_lldp_originals_for_the_next_agent) {
    // Without --keep-config an agent restores the NICs on a clean exit, but one that fails (here:
    // no LLDP peer within --wait) leaves them changed: its record must keep the originals, or
    // the next agent finds the flag "already" set and never restores it.
    Fixture f;
    f.cfg.wait_ns = 1000000;
    f.cfg.disable_fw_lldp = true;
    f.cfg.fw_lldp_state = f.tmp.path + "/fw-lldp-state";
    ethtool::PrivFlags ice{{"link-down-on-close", "fw-lldp-agent"}, 0x2};
    {
        auto eth = std::make_unique<FakeEthtool>();
        eth->drivers = {{"ens0", "ice"}};
        eth->flags["ens0"] = ice;
        FakeEthtool* raw = eth.get();
        agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());  // silent switch
        a.set_ethtool_ops(std::move(eth));
        CHECK_THROWS(a.run(-1));
        ice = raw->flags["ens0"];
    }
    CHECK_EQ(ice.bits, uint32_t(0));
    CHECK(read_file(f.cfg.fw_lldp_state) == std::optional<std::string>("ens0 priv 0x2\n"));
    auto eth = std::make_unique<FakeEthtool>();
    eth->drivers = {{"ens0", "ice"}};
    eth->flags["ens0"] = ice;
    FakeEthtool* raw = eth.get();
    Pipe stop;
    stop.fire();
    {
        agent::Agent b(f.cfg, f.ops, f.all_valid(), f.nm());
        b.set_ethtool_ops(std::move(eth));
        b.run(stop.fd[0]);
        CHECK(b.ready());
        // (the fake belongs to the agent: read it before the agent goes)
        CHECK_EQ(raw->flags["ens0"].bits, uint32_t(0x2));  // the true original, restored on the clean exit
    }
    CHECK(!path_exists(f.cfg.fw_lldp_state));
}

TEST(agent_keep_config_keeps_firmware_lldp_off_across_restarts_until_cleanup) {
    // keepConfigOnRestart + disableFirmwareLldp: a roll must not flip the NICs' firmware LLDP
    // back and forth (some drivers reset the port on a flip), and the originals must survive
    // agents that find the flag already set; --cleanup puts them back.
    Fixture f;
    f.cfg.keep_config = true;
    f.cfg.disable_fw_lldp = true;
    f.cfg.fw_lldp_dcbx_host = true;
    f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
    f.cfg.fw_lldp_state = f.tmp.path + "/fw-lldp-state";
    auto make_eth = [] {
        auto e = std::make_unique<FakeEthtool>();
        e->drivers = {{"ens0", "ice"}, {"ens1", "mlx5_core"}};
        return e;
    };
    ethtool::PrivFlags ice{{"link-down-on-close", "fw-lldp-agent"}, 0x2};  // firmware agent on
    uint8_t mlx = DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE;            // firmware DCBX
    std::vector<std::pair<std::string, uint32_t>> flag_sets;
    for (int run = 0; run < 2; ++run) {
        auto eth = make_eth();
        eth->flags["ens0"] = ice;
        eth->dcbx["ens1"] = mlx;
        FakeEthtool* raw = eth.get();
        Pipe stop;
        stop.fire();
        {
            agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
            a.set_ethtool_ops(std::move(eth));
            a.run(stop.fd[0]);
            CHECK(a.ready());
            ice = raw->flags["ens0"];  // what the NIC holds when the agent has gone
            mlx = raw->dcbx["ens1"];
            for (auto& x : raw->sets) flag_sets.push_back(x);
        }
        CHECK_EQ(ice.bits, uint32_t(0));                        // left off on exit
        CHECK_EQ(int(mlx), int(DCB_CAP_DCBX_HOST | DCB_CAP_DCBX_VER_CEE | DCB_CAP_DCBX_VER_IEEE));
        auto st = read_file(f.cfg.fw_lldp_state);
        CHECK(st && *st == "ens0 priv 0x2\nens1 dcbx 0x0c\n");  // the originals, also after run 2
    }
    CHECK_EQ(flag_sets.size(), size_t(1));  // set once, by the first agent; never flipped back
    {
        // keepConfigOnRestart turned off: the next agent finds the flags already set, takes the
        // originals from the record and restores those on exit (then the record is gone).
        agent::Config plain = f.cfg;
        plain.keep_config = false;
        auto eth = make_eth();
        eth->flags["ens0"] = ice;
        eth->dcbx["ens1"] = mlx;
        FakeEthtool* raw = eth.get();
        const std::string saved = *read_file(f.cfg.fw_lldp_state);
        Pipe stop;
        stop.fire();
        {
            agent::Agent a(plain, f.ops, f.all_valid(), f.nm());
            a.set_ethtool_ops(std::move(eth));
            a.run(stop.fd[0]);
            CHECK_EQ(raw->flags["ens0"].bits, uint32_t(0x2));  // (the fake goes with the agent)
            CHECK_EQ(int(raw->dcbx["ens1"]), 0x0c);
        }
        CHECK(!path_exists(f.cfg.fw_lldp_state));
        write_file_atomic(f.cfg.fw_lldp_state, saved);  // back to the kept state for the cleanup below
    }
    agent::Config c = f.cfg;
    c.cleanup = true;
    c.keep_config = false;
    auto eth = make_eth();
    eth->flags["ens0"] = ice;
    eth->dcbx["ens1"] = mlx;
    FakeEthtool* raw = eth.get();
    agent::Agent k(c, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
    k.set_ethtool_ops(std::move(eth));
    k.run(-1);
    CHECK_EQ(raw->flags["ens0"].bits, uint32_t(0x2));
    CHECK_EQ(int(raw->dcbx["ens1"]), 0x0c);
    CHECK(!path_exists(f.cfg.fw_lldp_state));
}

TEST(agent_node_lock_keeps_two_agents_of_one_kind_apart) {
    // The lock is an abstract unix socket: held by a live agent (here: by the test), a second
    // agent with the same name waits, then fails naming the cause; free, it is taken at once.
    Fixture f;
    f.cfg.keep_running = false;
    f.cfg.node_lock = "test-lock-" + std::to_string(::getpid());
    f.cfg.node_lock_wait_ns = 150000000;  // 150 ms
    sockaddr_un sa{};
    sa.sun_family = AF_UNIX;
    const std::string name = "netop-agent:" + f.cfg.node_lock;
    std::memcpy(sa.sun_path + 1, name.data(), name.size());
    int holder = ::socket(AF_UNIX, SOCK_STREAM, 0);
    CHECK(::bind(holder, reinterpret_cast<sockaddr*>(&sa), socklen_t(offsetof(sockaddr_un, sun_path) + 1 + name.size())) == 0);
    {
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        const int64_t t0 = mono_ns();
        bool threw = false;
        try {
            a.run(-1);
        } catch (const agent::AgentError& e) {
            threw = std::string(e.what()).find("holds the node lock") != std::string::npos;
        }
        CHECK(threw);
        CHECK(mono_ns() - t0 >= 140000000LL);
        CHECK(f.ops.addrs.empty());  // touched nothing
    }
    ::close(holder);  // the other agent exits (or dies): the kernel frees the name
    agent::Agent b(f.cfg, f.ops, f.all_valid(), f.nm());
    b.run(-1);
    CHECK_EQ(f.ops.addrs.size(), size_t(3));
    // Another name (a host-nic agent next to the scale-out one) never waits.
    agent::Config other = f.cfg;
    other.node_lock = f.cfg.node_lock + "-host-nic";
    agent::Agent c(other, f.ops, f.all_valid(), f.nm());
    const int64_t t1 = mono_ns();
    c.run(-1);
    CHECK(mono_ns() - t1 < 140000000LL);
}

TEST(agent_two_ports_describing_one_link_are_refused_and_named) {
    // ens2's switch port carries ens0's Port Description (copy-paste on the switch): ens0 keeps
    // the /30, ens2 is not configured, and the exit error says which NIC and why.
    for (bool pipeline : {true, false}) {
        Fixture f;
        f.cfg.keep_running = false;
        f.cfg.pipeline = pipeline;
        auto src = f.all_valid();
        src->frames["ens2"] = sw("02:aa:00:00:00:02", "no-alert 10.200.0.2/30");
        agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
        std::string err;
        try {
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        CHECK(err.find("Not all interfaces were configured (2/3).") != std::string::npos);
        CHECK(err.find("Not configured: ens2: its switch port describes 10.200.0.1/30, the link of ens0 too") !=
              std::string::npos);
        int on_ens0 = 0, on_ens2 = 0;
        for (auto& x : f.ops.addrs) {
            on_ens0 += x.ifindex == 10;
            on_ens2 += x.ifindex == 12;
        }
        CHECK_EQ(on_ens0, 1);
        CHECK_EQ(on_ens2, 0);
        auto st = read_file(f.cfg.status_file);
        CHECK(st && st->find("the link of ens0 too") != std::string::npos);
    }
}

TEST(agent_l3_start_configures_exactly_the_nics_with_a_unique_valid_port_description) {
    // Property of the L3 start (pipelined and not): six NICs, each with a random switch port --
    // a unique valid /30, an unusable Port Description, a copy of an earlier port's description,
    // or silence.  Exactly the NICs with a unique valid description (the first of a copied pair)
    // hold their /30 and nothing else; every other NIC holds nothing; the exit error counts them.
    uint64_t rng = 0xC0FFEE1234567ull;
    auto next = [&] {
        rng ^= rng << 13;
        rng ^= rng >> 7;
        rng ^= rng << 17;
        return rng;
    };
    int runs = 0, mismatches = 0;
    for (int round = 0; round < 24; ++round) {
        const bool pipeline = round % 2 == 0;
        Fixture f;
        f.cfg.keep_running = false;
        f.cfg.pipeline = pipeline;
        f.cfg.wait_ns = 50000000;
        std::vector<std::string> nics = {"ens0", "ens1", "ens2", "ens3", "ens4", "ens5"};
        for (int k = 3; k < 6; ++k) f.ops.add_link(nics[size_t(k)], 10 + k, strfmt("02:00:00:00:00:1%d", k).c_str(), true);
        f.cfg.interfaces = "ens0,ens1,ens2,ens3,ens4,ens5";
        auto src = std::make_unique<ScriptedLldp>();
        std::map<std::string, std::string> want;  // NIC -> the /30 it must hold
        std::map<std::string, std::string> desc_owner;
        for (int k = 0; k < 6; ++k) {
            const std::string& n = nics[size_t(k)];
            const std::string mac = strfmt("02:aa:00:00:00:%02d", k);
            int kind = int(next() % 4);
            if (kind == 2 && desc_owner.empty()) kind = 0;
            if (kind == 0) {
                const std::string d = strfmt("no-alert 10.%d.0.%d/30", 100 + round, 4 * k + 2);
                src->frames[n] = sw(mac.c_str(), d.c_str());
                want[n] = strfmt("10.%d.0.%d/30", 100 + round, 4 * k + 1);
                desc_owner[d] = n;
            } else if (kind == 1) {
                src->frames[n] = sw(mac.c_str(), "no-alert not-an-address");
            } else if (kind == 2) {
                auto it = desc_owner.begin();
                std::advance(it, long(next() % desc_owner.size()));
                src->frames[n] = sw(mac.c_str(), it->first.c_str());
            }  // kind 3: silent
        }
        agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
        std::string err;
        try {
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        ++runs;
        bool ok = true;
        for (int k = 0; k < 6; ++k) {
            const std::string& n = nics[size_t(k)];
            std::vector<std::string> have;
            for (const auto& x : f.ops.addrs)
                if (x.ifindex == 10 + k) have.push_back(x.prefix().str());
            const std::vector<std::string> expect = want.count(n) ? std::vector<std::string>{want[n]}
                                                                  : std::vector<std::string>{};
            if (have != expect) ok = false;
        }
        if (want.size() == 6)
            ok = ok && err.empty();
        else if (want.empty())
            ok = ok && err.find("No LLDP peers with a /30 Port Description were found") == 0;
        else
            ok = ok && err.find(strfmt("Not all interfaces were configured (%zu/6).", want.size())) == 0;
        if (!ok) {
            if (!mismatches) fprintf(stderr, "round %d (pipeline %d): %s\n", round, pipeline, err.c_str());
            ++mismatches;
        }
    }
    CHECK_EQ(mismatches, 0);
    CHECK_EQ(runs, 24);
}

TEST(agent_min_link_speed_refuses_a_nic_that_came_up_slow) {
    // ens1 negotiated 200G on a 400G fabric: left unconfigured (L3) and named; ens2 reports no
    // speed (allowed, warned); L2 fails the start with the same reason.
    for (const char* mode : {"L3", "L2"}) {
        Fixture f;
        f.cfg.mode = mode;
        f.cfg.keep_running = false;
        f.cfg.min_link_speed_mbps = 400000;
        f.cfg.sysfs_root = f.tmp.path + "/sys";
        f.tmp.write("sys/class/net/ens0/speed", "400000\n");
        f.tmp.write("sys/class/net/ens1/speed", "200000\n");
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        std::string err;
        try {
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        const std::string why = "ens1: link negotiated at 200 Gb/s, below the required 400 Gb/s";
        CHECK(err.find(why) != std::string::npos);
        if (std::string(mode) == "L3") {
            CHECK(err.find("Not all interfaces were configured (2/3).") != std::string::npos);
            for (auto& x : f.ops.addrs) CHECK(x.ifindex != 11);
        } else {
            CHECK(err.find("1 NIC(s) below the required link speed") != std::string::npos);
        }
        auto st = read_file(f.cfg.status_file);
        CHECK(st && st->find("\"speed_mbps\":200000") != std::string::npos);
    }
    CHECK_EQ(topo::netdev_speed_mbps("/nonexistent", "ens0"), -1);
}

TEST(lldp_max_frame_size_tlv_roundtrip) {
    auto f = lldp::make_switch_frame(*MacAddr::parse("02:aa:00:00:00:01"), "tor", "p1", "no-alert 10.200.0.6/30");
    CHECK(!f.max_frame_size());
    f.set_max_frame_size(9216);
    f.set_max_frame_size(1518);  // replaces, never duplicates
    auto bytes = lldp::encode(f);
    auto d = lldp::decode(bytes.data(), bytes.size());
    CHECK(d && d->max_frame_size() && *d->max_frame_size() == 1518);
    CHECK(d && d->org.size() == 1);
}

TEST(agent_switch_port_with_a_smaller_max_frame_than_the_mtu_is_refused) {
    // MTU 9000: ens1's switch port still accepts only 1518-byte frames (jumbo not enabled on
    // it) -> refused and named; 9216 and "not advertised" pass.  At MTU 1500, 1518 is enough.
    for (int mtu : {9000, 1500}) {
        Fixture f;
        f.cfg.keep_running = false;
        f.cfg.mtu = mtu;
        auto src = f.all_valid();
        src->frames["ens0"].set_max_frame_size(9216);
        src->frames["ens1"].set_max_frame_size(1518);
        agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
        std::string err;
        try {
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        if (mtu == 9000) {
            CHECK(err.find("Not configured: ens1: its switch port accepts frames up to 1518 bytes, but MTU 9000 needs "
                           "9018") != std::string::npos);
            auto st = read_file(f.cfg.status_file);
            CHECK(st && st->find("\"peer_max_frame\":1518") != std::string::npos);
        } else {
            CHECK(err.empty());
            CHECK_EQ(f.ops.addrs.size(), size_t(3));
        }
    }
    Fixture g;  // the check can be turned off
    g.cfg.keep_running = false;
    g.cfg.mtu = 9000;
    g.cfg.check_peer_mtu = false;
    auto src = g.all_valid();
    src->frames["ens1"].set_max_frame_size(1518);
    agent::Agent b(g.cfg, g.ops, std::move(src), g.nm());
    b.run(-1);
    CHECK_EQ(g.ops.addrs.size(), size_t(3));
}

TEST(agent_announcement_carries_the_hosts_max_frame_size) {
    auto f = agent::make_node_frame("node-1", "ens0", *MacAddr::parse("02:00:00:00:00:10"), "0000:05:00.0", 120, 9000);
    CHECK(f.max_frame_size() && *f.max_frame_size() == 9018);
    CHECK(!agent::make_node_frame("node-1", "ens0", *MacAddr::parse("02:00:00:00:00:10"), "", 0, 9000).max_frame_size());
    CHECK(!agent::make_node_frame("node-1", "ens0", *MacAddr::parse("02:00:00:00:00:10"), "").max_frame_size());
}

namespace {
// Host NICs for rdma discovery: three PCI NICs on their own root ports (no GPU next to them),
// each with an RDMA device, netdevs named like the Fixture's links.
void host_nic_sysfs(const TmpDir& t) {
    int k = 0;
    for (const char* name : {"ens0", "ens1", "ens2"}) {
        const std::string bdf = strfmt("0000:%02x:00.0", 0x40 + k);
        const std::string dev = strfmt("devices/pci0000:%02x/0000:%02x:01.1/%s", 0x40 + k, 0x40 + k, bdf.c_str());
        t.write(dev + "/vendor", "0x15b3\n");
        t.write(dev + "/device", "0x1021\n");
        t.mkdir("bus/pci/drivers/mlx5_core");
        t.symlink("bus/pci/drivers/mlx5_core", dev + "/driver");
        t.write(dev + "/net/" + name + "/address", strfmt("02:00:00:00:00:1%d\n", k));
        t.symlink(dev + "/net/" + name, std::string("class/net/") + name);
        t.mkdir(dev + "/infiniband/mlx5_" + std::to_string(k));
        ++k;
    }
}

nl::RouteSpec route(int ifindex, const char* dst, const char* gw, uint8_t proto) {
    nl::RouteSpec r;
    r.ifindex = ifindex;
    r.dst = *Ipv4Prefix::parse(dst);
    if (gw) r.gateway = *Ipv4::parse(gw);
    r.protocol = proto;
    return r;
}
}  // namespace

TEST(agent_rdma_discovery_leaves_the_nodes_own_nics_alone) {
    // A default host-nic policy (rdma discovery, default drivers): ens0 carries the default route
    // and ens1 holds the node's 192.168.1.5/24, so only ens2 is taken; with a DHCP route through
    // ens2 as well (variant 1) nothing is left, and the error lists why for each NIC.
    for (int variant : {0, 1}) {
        Fixture f;
        f.cfg.mode = "L2";
        f.cfg.keep_running = false;
        f.cfg.interfaces = "";
        f.cfg.discovery.mode = topo::DiscoveryMode::Rdma;
        TmpDir sys;
        host_nic_sysfs(sys);
        f.cfg.sysfs_root = sys.path;
        f.ops.routes.push_back(route(10, "0.0.0.0/0", "192.168.0.1", RTPROT_DHCP));
        f.ops.addrs.push_back(nl::AddrInfo{11, AF_INET, *Ipv4::parse("192.168.1.5"), *Ipv4::parse("192.168.1.5"), 24, 0, ""});
        if (variant == 1) f.ops.routes.push_back(route(12, "172.16.0.0/12", "172.16.0.1", RTPROT_DHCP));
        agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
        std::string err;
        try {
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        if (variant == 0) {
            CHECK(err.empty());
            CHECK_EQ(a.nics().size(), size_t(1));
            CHECK_EQ(a.nics()[0].ifname, std::string("ens2"));
            CHECK_EQ(f.ops.links["ens2"].mtu, 1500);
            CHECK(f.ops.links["ens2"].flags & IFF_UP);
        } else {
            CHECK(err.find("No interfaces found (left alone: ") == 0);
            CHECK(err.find("ens2: the node's own NIC: it has the route 172.16.0.0/12 (protocol dhcp)") != std::string::npos);
        }
        CHECK(err.empty() == (variant == 0));
        // The node's NICs kept everything: address, routes, MTU, admin state.
        CHECK_EQ(f.ops.addrs.size(), size_t(1));
        CHECK(!(f.ops.links["ens0"].flags & IFF_UP));  // was down, never brought up
        CHECK_EQ(f.ops.calls["addr_del"], 0);
        auto ex = a.excluded();
        CHECK_EQ(ex.size(), size_t(variant == 0 ? 2 : 3));
        CHECK_EQ(ex[0].first, std::string("ens0"));
        CHECK_EQ(ex[0].second, std::string("the node's own NIC: it carries the node's default route"));
        CHECK_EQ(ex[1].second, std::string("the node's own NIC: it holds 192.168.1.5/24, an address the agent never "
                                           "assigns (it only uses /30s)"));
        if (variant == 0) {
            auto st = read_file(f.cfg.status_file);
            CHECK(st && st->find("\"excluded\":\"ens0: the node's own NIC: it carries the node's default route; "
                                 "ens1: ") != std::string::npos);
        }
    }
}

TEST(agent_rdma_discovery_leaves_bond_ports_and_vlan_parents_the_node_uses_alone) {
    // Stacked devices: ens0 is a port of bond0; ens1 carries the VLAN ens1.100 with the node's
    // 10.0.100.5/24 (a management VLAN on a RoCE port); ens2 carries ens2.200, which holds nothing.
    // Variant 0: bond0 has the default route; variant 1: it has none (a port is still not ours).
    // Named explicitly, the bond port under the default route is refused like the uplink itself.
    for (int variant : {0, 1}) {
        Fixture f;
        f.cfg.mode = "L2";
        f.cfg.keep_running = false;
        f.cfg.interfaces = "";
        f.cfg.discovery.mode = topo::DiscoveryMode::Rdma;
        TmpDir sys;
        host_nic_sysfs(sys);
        f.cfg.sysfs_root = sys.path;
        f.ops.add_link("bond0", 20, "02:00:00:00:00:20", true);
        f.ops.add_link("ens1.100", 21, "02:00:00:00:00:21", true);
        f.ops.add_link("ens2.200", 22, "02:00:00:00:00:22", true);
        f.ops.links["ens0"].master = 20;
        sys.mkdir("devices/virtual/net/bond0");
        sys.symlink("devices/virtual/net/bond0", "class/net/ens0/upper_bond0");
        sys.symlink("devices/virtual/net/ens1.100", "class/net/ens1/upper_ens1.100");
        sys.symlink("devices/virtual/net/ens2.200", "class/net/ens2/upper_ens2.200");
        CHECK(topo::netdev_uppers(sys.path, "ens0") == std::vector<std::string>{"bond0"});
        if (variant == 0) f.ops.routes.push_back(route(20, "0.0.0.0/0", "192.168.0.1", RTPROT_DHCP));
        f.ops.addrs.push_back(nl::AddrInfo{21, AF_INET, *Ipv4::parse("10.0.100.5"), *Ipv4::parse("10.0.100.5"), 24, 0, ""});
        agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
        a.run(-1);
        CHECK_EQ(a.nics().size(), size_t(1));
        CHECK_EQ(a.nics()[0].ifname, std::string("ens2"));
        auto ex = a.excluded();
        CHECK_EQ(ex.size(), size_t(2));
        CHECK_EQ(ex[0].second, std::string(variant == 0 ? "the node's own NIC: it carries the node's default route via bond0"
                                                        : "the node's own NIC: it is a port of bond0 (a bond, bridge, "
                                                          "team or VRF: the node configures the master, not its ports)"));
        CHECK_EQ(ex[1].second, std::string("the node's own NIC: it carries ens1.100, which holds 10.0.100.5/24, an "
                                           "address the agent never assigns (it only uses /30s)"));
        const std::string m = a.render_metrics();
        CHECK(m.find(std::string("netop_agent_nic_left_alone{nic=\"ens0\",reason=\"") +
                     (variant == 0 ? "default_route" : "bond_or_bridge_port") + "\"} 1") != std::string::npos);
        CHECK(m.find("netop_agent_nic_left_alone{nic=\"ens1\",reason=\"stacked_device\"} 1") != std::string::npos);
        CHECK_EQ(f.ops.links["ens0"].mtu, 1500);
        CHECK_EQ(f.ops.links["ens1"].mtu, 1500);

        if (variant == 0) {  // named: refused, with the path
            Fixture g;
            g.cfg.interfaces = "ens0";
            g.cfg.sysfs_root = sys.path;
            g.ops.add_link("bond0", 20, "02:00:00:00:00:20", true);
            g.ops.links["ens0"].master = 20;
            g.ops.routes.push_back(route(20, "0.0.0.0/0", "192.168.0.1", RTPROT_DHCP));
            agent::Agent b(g.cfg, g.ops, g.all_valid(), g.nm());
            std::string err;
            try {
                b.run(-1);
            } catch (const agent::AgentError& e) {
                err = e.what();
            }
            CHECK(err.find("Refusing to configure ens0 via bond0: the node's default route leaves through it") == 0);
            CHECK_EQ(g.ops.calls["addr_del"], 0);

            // Without sysfs upper links (the master from rtnetlink alone): the same refusal.
            Fixture h;
            h.cfg.interfaces = "ens0";
            h.ops.add_link("br0", 30, "02:00:00:00:00:30", true);
            h.ops.links["ens0"].master = 30;
            h.ops.routes.push_back(route(30, "0.0.0.0/0", "192.168.0.1", RTPROT_DHCP));
            agent::Agent c(h.cfg, h.ops, h.all_valid(), h.nm());
            err.clear();
            try {
                c.run(-1);
            } catch (const agent::AgentError& e) {
                err = e.what();
            }
            CHECK(err.find("Refusing to configure ens0 via br0: ") == 0);
        }
    }
}

TEST(agent_rdma_discovery_leaves_a_nic_with_a_global_ipv6_address_alone) {
    // An IPv6-only storage network on ens1 (a ULA address, no default route): the node's.  A
    // link-local address (every up NIC has one) does not count.
    Fixture f;
    f.cfg.mode = "L2";
    f.cfg.keep_running = false;
    f.cfg.interfaces = "";
    f.cfg.discovery.mode = topo::DiscoveryMode::Rdma;
    TmpDir sys;
    host_nic_sysfs(sys);
    f.cfg.sysfs_root = sys.path;
    nl::AddrInfo ula{};
    ula.ifindex = 11;
    ula.family = AF_INET6;
    ula.address6 = "fd00:77::5";
    ula.prefixlen = 64;
    ula.scope = RT_SCOPE_UNIVERSE;
    nl::AddrInfo ll = ula;
    ll.ifindex = 12;
    ll.address6 = "fe80::2";
    ll.scope = RT_SCOPE_LINK;
    f.ops.addrs.push_back(ula);
    f.ops.addrs.push_back(ll);
    agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
    a.run(-1);
    std::vector<std::string> got;
    for (const auto& n : a.nics()) got.push_back(n.ifname);
    CHECK(got == (std::vector<std::string>{"ens0", "ens2"}));
    auto ex = a.excluded();
    CHECK_EQ(ex.size(), size_t(1));
    CHECK_EQ(ex[0].second, std::string("the node's own NIC: it holds fd00:77::5/64, an IPv6 address the agent never assigns"));
}

TEST(agent_restore_mtu_puts_each_nics_mtu_back_on_a_clean_exit_only) {
    // --restore-mtu (host-nic policies): MTU 9000 while the agent runs, each NIC's own MTU (1500,
    // 4200) back after a clean exit; with --keep-config the next agent adopts the NICs as they are.
    for (bool keep : {false, true}) {
        Fixture f;
        f.cfg.mode = "L2";
        f.cfg.mtu = 9000;
        f.cfg.restore_mtu = true;
        f.cfg.keep_config = keep;
        f.ops.links["ens1"].mtu = 4200;
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
        bool jumbo = false;
        a.on_monitor_tick = [&](int) {
            jumbo = f.ops.links["ens0"].mtu == 9000 && f.ops.links["ens1"].mtu == 9000;
            stop.fire();
        };
        a.run(stop.fd[0]);
        CHECK(jumbo);
        CHECK_EQ(f.ops.links["ens0"].mtu, keep ? 9000 : 1500);
        CHECK_EQ(f.ops.links["ens1"].mtu, keep ? 9000 : 4200);
    }
}

TEST(agent_mtu_state_keeps_the_original_mtu_across_keep_config_restarts_for_the_cleanup) {
    // Host NICs with keepConfigOnRestart: the first agent records ens1's own MTU (4200) before it
    // sets 9000; a restarted agent finds 9000 on the NIC but keeps the recorded 4200; the cleanup
    // Job puts 4200 back and removes the record.  Without --keep-config a clean exit does it.
    Fixture f;
    f.cfg.mode = "L2";
    f.cfg.mtu = 9000;
    f.cfg.restore_mtu = true;
    f.cfg.keep_config = true;
    f.cfg.keep_running = false;
    f.cfg.mtu_state = f.tmp.path + "/mtu-state";
    f.ops.links["ens1"].mtu = 4200;
    for (int restart = 0; restart < 2; ++restart) {
        agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
        a.run(-1);
        CHECK_EQ(f.ops.links["ens1"].mtu, 9000);
        auto st = read_file(f.cfg.mtu_state);
        CHECK(st && *st == "ens0 1500\nens1 4200\nens2 1500\n");
    }
    agent::Config c = f.cfg;
    c.cleanup = true;
    {
        agent::Agent a(c, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
        a.run(-1);
    }
    CHECK_EQ(f.ops.links["ens1"].mtu, 4200);
    CHECK_EQ(f.ops.links["ens0"].mtu, 1500);
    CHECK(!path_exists(f.cfg.mtu_state));

    Fixture g;  // no --keep-config: the clean exit (SIGTERM) restores and leaves no record
    g.cfg.mode = "L2";
    g.cfg.mtu = 9000;
    g.cfg.restore_mtu = true;
    g.cfg.mtu_state = g.tmp.path + "/mtu-state";
    {
        Pipe stop;
        stop.fire();
        agent::Agent a(g.cfg, g.ops, std::make_unique<ScriptedLldp>(), g.nm());
        a.run(stop.fd[0]);
        CHECK(a.ready());
    }
    CHECK_EQ(g.ops.links["ens0"].mtu, 1500);
    CHECK(!path_exists(g.cfg.mtu_state));
}

TEST(agent_link_state_keeps_the_original_down_state_across_a_crash_for_the_last_exit) {
    // ens0 and ens2 are down before any agent; the first agent brings them up and dies without
    // cleaning up (here: a --keep-config exit, which leaves the links up just the same).  The next
    // agent finds them up, but the record says down: its clean exit takes them down again and
    // removes the record.  ens1 was up before any agent and stays up.  --cleanup does the same
    // from the record alone.
    for (bool via_cleanup : {false, true}) {
        Fixture f;
        f.cfg.mode = "L2";
        f.cfg.keep_running = false;
        f.cfg.link_state = f.tmp.path + "/link-state";
        {
            agent::Config c = f.cfg;
            c.keep_config = true;
            agent::Agent a(c, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
            a.run(-1);
        }
        CHECK(f.ops.links["ens0"].flags & IFF_UP);
        CHECK(read_file(f.cfg.link_state) == std::optional<std::string>("ens0 down\nens1 up\nens2 down\n"));
        if (via_cleanup) {
            agent::Config c = f.cfg;
            c.cleanup = true;
            agent::Agent a(c, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
            a.run(-1);
        } else {
            agent::Config c = f.cfg;
            c.keep_running = true;
            Pipe stop;
            stop.fire();
            agent::Agent a(c, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
            a.run(stop.fd[0]);
            CHECK(a.ready());
        }
        CHECK(!(f.ops.links["ens0"].flags & IFF_UP));
        CHECK(!(f.ops.links["ens2"].flags & IFF_UP));
        CHECK(f.ops.links["ens1"].flags & IFF_UP);
        CHECK(!path_exists(f.cfg.link_state));
    }
    Fixture g;  // without the record: the restarted agent takes "up" for the original (the reference)
    g.cfg.mode = "L2";
    {
        agent::Config c = g.cfg;
        c.keep_config = true;
        c.keep_running = false;
        agent::Agent a(c, g.ops, std::make_unique<ScriptedLldp>(), g.nm());
        a.run(-1);
    }
    {
        Pipe stop;
        stop.fire();
        agent::Agent a(g.cfg, g.ops, std::make_unique<ScriptedLldp>(), g.nm());
        a.run(stop.fd[0]);
    }
    CHECK(g.ops.links["ens0"].flags & IFF_UP);
}

TEST(agent_rdma_discovery_keeps_the_agents_own_l3_config) {
    // A host NIC an earlier (keep-config) agent addressed: its /30, the kernel /30 route, the /16
    // via the switch end and the rail table are the agent's, so the NIC is still a host NIC.
    Fixture f;
    f.cfg.keep_running = false;
    f.cfg.interfaces = "";
    f.cfg.discovery.mode = topo::DiscoveryMode::Rdma;
    TmpDir sys;
    host_nic_sysfs(sys);
    f.cfg.sysfs_root = sys.path;
    f.ops.addr_add(10, *Ipv4Prefix::parse("10.200.0.1/30"));
    f.ops.routes.push_back(route(10, "10.200.0.0/16", "10.200.0.2", RTPROT_BOOT));
    auto rail = route(10, "10.200.0.0/16", "10.200.0.2", agent::kRailProtocol);
    rail.table = 100;
    f.ops.routes.push_back(rail);
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    CHECK_EQ(a.nics().size(), size_t(3));
    CHECK(a.excluded().empty());
}

TEST(agent_refuses_a_nic_that_carries_the_default_route_in_every_mode) {
    // Named explicitly (--interfaces) or discovered, L2 or L3, multipath or not: the uplink is
    // never flushed or re-MTUed; the error names it.  A dry run reports it instead.
    for (const char* mode : {"L3", "L2"})
        for (bool multipath : {false, true}) {
            Fixture f;
            f.cfg.mode = mode;
            f.cfg.mtu = 9000;
            f.ops.addrs.push_back(nl::AddrInfo{11, AF_INET, *Ipv4::parse("192.168.1.5"), *Ipv4::parse("192.168.1.5"), 24, 0, ""});
            auto def = route(multipath ? 0 : 11, "0.0.0.0/0", "192.168.1.1", RTPROT_STATIC);
            if (multipath) def.nexthops = {13, 11};
            f.ops.routes.push_back(def);
            agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
            std::string err;
            try {
                a.run(-1);
            } catch (const agent::AgentError& e) {
                err = e.what();
            }
            CHECK(err.find("Refusing to configure ens1: the node's default route leaves through it") == 0);
            CHECK_EQ(f.ops.addrs.size(), size_t(1));
            CHECK_EQ(f.ops.links["ens1"].mtu, 1500);
            CHECK_EQ(f.ops.calls["link_set_up"], 0);
        }
    Fixture d;
    d.cfg.dry_run = true;
    d.ops.routes.push_back(route(11, "0.0.0.0/0", "192.168.1.1", RTPROT_DHCP));
    agent::Agent a(d.cfg, d.ops, d.all_valid(), d.nm());
    a.run(-1);
    CHECK_EQ(a.excluded().size(), size_t(1));
    CHECK_EQ(a.excluded()[0].second, std::string("carries the node's default route (refused)"));
    // Failing to read the routes is not taken for "no uplink".
    Fixture g;
    g.ops.fail.insert("route_list");
    agent::Agent b(g.cfg, g.ops, g.all_valid(), g.nm());
    std::string err;
    try {
        b.run(-1);
    } catch (const agent::AgentError& e) {
        err = e.what();
    }
    CHECK(err.find("Cannot read the node's routes") == 0);
}

TEST(agent_configures_a_nic_whose_default_route_is_only_in_a_policy_routing_table) {
    // multi-rail RoCE nodes give each NIC its own source-routing table with a default
    // route in it ("from 192.168.1.0/24 lookup 101").  Only selective rules reach that table:
    // it is not the node's uplink, and the NIC is configured.  A default route in a table that
    // a rule selecting nothing reaches (main) still is.  Unreadable rules: every table counts.
    auto rule = [](uint32_t table, uint32_t prio, const char* src) {
        nl::RuleSpec r;
        r.table = table;
        r.priority = prio;
        if (src) {
            r.src = *Ipv4Prefix::parse(src);
            r.selective = true;
        }
        return r;
    };
    for (int variant : {0, 1, 2}) {
        Fixture f;
        f.cfg.mode = "L3";
        f.cfg.keep_running = false;
        f.ops.rules = {rule(RT_TABLE_LOCAL, 0, nullptr), rule(101, 100, "192.168.1.0/24"),
                       rule(RT_TABLE_MAIN, 32766, nullptr), rule(RT_TABLE_DEFAULT, 32767, nullptr)};
        auto def = route(11, "0.0.0.0/0", "192.168.1.1", RTPROT_STATIC);
        def.table = variant == 1 ? uint32_t(RT_TABLE_MAIN) : 101u;
        f.ops.routes.push_back(def);
        if (variant == 2) f.ops.fail.insert("rule_list");
        std::string err;
        try {
            agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        if (variant == 0) {
            CHECK(f.ops.default_route_links().empty());
            CHECK(f.ops.policy_default_routes() == (std::vector<std::pair<int, uint32_t>>{{11, 101}}));
            CHECK_EQ(err, std::string());
            CHECK_EQ(f.ops.addrs.size(), size_t(3));  // every NIC configured, ens1 too
        } else {
            CHECK(err.find("Refusing to configure ens1: the node's default route leaves through it") == 0);
            CHECK_EQ(f.ops.calls["link_set_up"], 0);
        }
    }
}

TEST(agent_nic_lock_gives_every_nic_one_owner) {
    // Another agent (a host-nic policy naming a rail, say) holds ens1: this agent, whatever its
    // label file, waits, then fails naming the NIC, having changed nothing; once the holder is
    // gone it proceeds.
    Fixture f;
    f.cfg.keep_running = false;
    f.cfg.nic_locks = true;
    f.cfg.node_lock_wait_ns = 150000000;  // 150 ms
    f.cfg.interfaces = "ens0,ens1,ens2";
    // Per-process names: the abstract namespace is node (network namespace) wide.
    const std::string name = "netop-nic:ens1";
    sockaddr_un sa{};
    sa.sun_family = AF_UNIX;
    std::memcpy(sa.sun_path + 1, name.data(), name.size());
    int holder = ::socket(AF_UNIX, SOCK_STREAM, 0);
    const bool bound =
        ::bind(holder, reinterpret_cast<sockaddr*>(&sa), socklen_t(offsetof(sockaddr_un, sun_path) + 1 + name.size())) == 0;
    CHECK(bound);
    {
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        std::string err;
        try {
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        CHECK(err.find("Another agent holds NIC 'ens1' (its NIC lock)") == 0);
        CHECK(f.ops.addrs.empty());
        CHECK_EQ(f.ops.calls["link_set_up"], 0);
    }
    ::close(holder);
    agent::Agent b(f.cfg, f.ops, f.all_valid(), f.nm());
    b.run(-1);
    CHECK_EQ(f.ops.addrs.size(), size_t(3));
}

TEST(agent_l2_waits_for_carrier_and_labels_only_when_every_nic_has_a_link) {
    // L2 starts with ens1's cable unplugged: no label, the reason names it (status.json and the
    // readiness probe's file); the carrier comes and the monitor publishes the label.
    Fixture f;
    f.cfg.mode = "L2";
    f.cfg.monitor_tick_ns = 1000000;
    f.ops.no_carrier = {"ens1"};
    f.ops.links["ens1"].flags &= ~unsigned(IFF_LOWER_UP);
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
    bool unlabelled = false, reason = false, status = false, labelled = false, dark_metric = false, lit_metric = false;
    a.on_monitor_tick = [&](int tick) {
        if (tick == 1) {
            dark_metric = a.render_metrics().find("netop_agent_nic_carrier{nic=\"ens1\"} 0\n") != std::string::npos;
            unlabelled = !path_exists(f.cfg.labels.path());
            auto why = read_file(agent::reason_path(f.cfg.status_file));
            reason = why && *why == "ens1: no carrier (check the cable, the switch port and the optic)\n";
            auto st = read_file(f.cfg.status_file);
            status = st && st->find("\"ready\":false") != std::string::npos &&
                     st->find("\"no_carrier\":true") != std::string::npos;
            f.ops.set_carrier("ens1", true);
        } else if (tick == 3) {
            labelled = path_exists(f.cfg.labels.path()) && !path_exists(agent::reason_path(f.cfg.status_file));
            lit_metric = a.render_metrics().find("netop_agent_nic_carrier{nic=\"ens1\"} 1\n") != std::string::npos;
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(dark_metric);
    CHECK(lit_metric);
    CHECK(unlabelled);
    CHECK(reason);
    CHECK(status);
    CHECK(labelled);
    // Without the monitor nothing would notice the carrier later: the start fails, naming it.
    Fixture g;
    g.cfg.mode = "L2";
    g.cfg.keep_running = false;
    g.ops.no_carrier = {"ens2"};
    agent::Agent b(g.cfg, g.ops, std::make_unique<ScriptedLldp>(), g.nm());
    std::string err;
    try {
        b.run(-1);
    } catch (const agent::AgentError& e) {
        err = e.what();
    }
    CHECK(err.find("Not all interfaces have a link (2/3). No carrier: ens2") == 0);
    CHECK(!path_exists(g.cfg.labels.path()));
}

TEST(agent_l2_checks_the_link_speed_when_the_carrier_comes_and_after_a_flap) {
    // L2 with the monitor, 400G required.  ens1 has no cable at the start (the kernel reports no
    // speed); when its carrier comes it has negotiated 200G: still no label, the speed named.  The
    // port flaps and comes back at 400G: the label follows.  A NIC that is slow from the start
    // keeps the node unlabelled the same way instead of failing the start.
    Fixture f;
    f.cfg.mode = "L2";
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.min_link_speed_mbps = 400000;
    f.cfg.sysfs_root = f.tmp.path + "/sys";
    f.tmp.write("sys/class/net/ens0/speed", "400000\n");
    f.tmp.write("sys/class/net/ens1/speed", "-1\n");
    f.tmp.write("sys/class/net/ens2/speed", "400000\n");
    f.ops.no_carrier = {"ens1"};
    f.ops.links["ens1"].flags &= ~unsigned(IFF_LOWER_UP);
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
    auto reason = [&] { return read_file(agent::reason_path(f.cfg.status_file)).value_or(""); };
    bool dark = false, slow = false, labelled = false;
    a.on_monitor_tick = [&](int tick) {
        if (tick == 1) {
            dark = !path_exists(f.cfg.labels.path()) && reason().find("ens1: no carrier") == 0;
            f.tmp.write("sys/class/net/ens1/speed", "200000\n");
            f.ops.set_carrier("ens1", true);
        } else if (tick == 3) {
            slow = !path_exists(f.cfg.labels.path()) &&
                   reason().find("ens1: link negotiated at 200 Gb/s, below the required 400 Gb/s") == 0;
            f.ops.set_carrier("ens1", false);
        } else if (tick == 5) {
            f.tmp.write("sys/class/net/ens1/speed", "400000\n");
            f.ops.set_carrier("ens1", true);
        } else if (tick == 7) {
            labelled = path_exists(f.cfg.labels.path()) && !path_exists(agent::reason_path(f.cfg.status_file));
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(dark);
    CHECK(slow);
    CHECK(labelled);

    Fixture g;
    g.cfg.mode = "L2";
    g.cfg.monitor_tick_ns = 1000000;
    g.cfg.min_link_speed_mbps = 400000;
    g.cfg.sysfs_root = g.tmp.path + "/sys";
    g.tmp.write("sys/class/net/ens2/speed", "100000\n");
    Pipe stop2;
    agent::Agent b(g.cfg, g.ops, std::make_unique<ScriptedLldp>(), g.nm());
    std::string why;
    b.on_monitor_tick = [&](int) {
        why = read_file(agent::reason_path(g.cfg.status_file)).value_or("");
        stop2.fire();
    };
    b.run(stop2.fd[0]);
    CHECK(why.find("ens2: link negotiated at 100 Gb/s") == 0);
    CHECK(!path_exists(g.cfg.labels.path()));
}

TEST(agent_l2_label_follows_a_random_sequence_of_flaps_and_speed_changes) {
    // Property: under any sequence of cable pulls, re-plugs and speed renegotiations, the L2 label
    // is published exactly when every NIC is ready, where a NIC is ready when it has carrier and
    // had the required speed when its carrier last came (the speed is read at that moment, as a
    // port renegotiates when its link comes up).  The readiness probe's reason file exists exactly
    // when the label does not.  200 random steps for each of three fixed seeds.
    for (uint64_t seed : {0x9E3779B97F4A7C15ull, 0x1234567887654321ull, 0xDEADBEEFCAFEBABEull}) {
        Fixture f;
        f.cfg.mode = "L2";
        f.cfg.monitor_tick_ns = 1000000;
        f.cfg.min_link_speed_mbps = 400000;
        f.cfg.sysfs_root = f.tmp.path + "/sys";
        const std::vector<std::string> nics = {"ens0", "ens1", "ens2"};
        std::map<std::string, bool> carrier, ready;
        std::map<std::string, int64_t> speed;
        for (const auto& n : nics) {
            carrier[n] = ready[n] = true;
            speed[n] = 400000;
            f.tmp.write("sys/class/net/" + n + "/speed", "400000\n");
        }
        uint64_t rng = seed;
        auto next = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, std::make_unique<ScriptedLldp>(), f.nm());
        int checked = 0, mismatches = 0, labelled_states = 0;
        std::string first_bad;
        a.on_monitor_tick = [&](int tick) {
            if (tick % 2 == 0) {  // the previous step has been processed: check
                bool want = std::all_of(nics.begin(), nics.end(), [&](const std::string& n) { return ready[n]; });
                bool label = path_exists(f.cfg.labels.path());
                bool reason = path_exists(agent::reason_path(f.cfg.status_file));
                ++checked;
                labelled_states += want;
                if (label != want || reason == want) {
                    if (!mismatches) first_bad = strfmt("tick %d: want %d label %d reason %d", tick, want, label, reason);
                    ++mismatches;
                }
                if (tick >= 400) stop.fire();
                return;
            }
            const std::string& n = nics[next() % nics.size()];
            if (next() % 4 == 0) {  // the port renegotiates (takes effect at the next link-up)
                speed[n] = next() % 4 ? 400000 : 200000;
                f.tmp.write("sys/class/net/" + n + "/speed", std::to_string(speed[n]) + "\n");
            } else {
                carrier[n] = !carrier[n];
                ready[n] = carrier[n] && speed[n] >= 400000;
                f.ops.set_carrier(n, carrier[n]);
            }
        };
        a.run(stop.fd[0]);
        if (mismatches) fprintf(stderr, "seed %llx, %s\n", (unsigned long long)seed, first_bad.c_str());
        CHECK_EQ(mismatches, 0);
        CHECK_EQ(checked, 201);
        CHECK(labelled_states > 0 && labelled_states < checked);  // the sequence visits both states
    }
}

TEST(agent_l3_label_and_addresses_follow_random_flaps_and_re_addressing) {
    // Property (L3 with the monitor): under any sequence of cable pulls, re-plugs and switch-port
    // re-addressing (a new /30 in the Port Description), the label is published exactly when every
    // NIC has carrier, and every NIC with carrier holds exactly the /30 its switch port currently
    // describes (peer ^ 3).  Frames only arrive while a NIC has carrier.  Three seeds.
    for (uint64_t seed : {0xA5A5A5A55A5A5A5Aull, 0x0123456789ABCDEFull, 0x7777000011112222ull}) {
        Fixture f;
        f.cfg.monitor_tick_ns = 1000000;
        f.cfg.lldp_tx_interval_ns = 3600LL * 1000000000LL;
        const std::vector<std::string> nics = {"ens0", "ens1", "ens2"};
        std::map<std::string, int> idx = {{"ens0", 10}, {"ens1", 11}, {"ens2", 12}};
        std::map<std::string, bool> carrier;
        std::map<std::string, int> host;  // the switch end is 10.20k.0.(4*host+2), ours +1 (^3)
        auto src = f.all_valid();
        ScriptedLldp* lldp_src = src.get();
        std::map<std::string, lldp::Frame> frames;
        auto describe = [&](const std::string& n) {
            const int k = int(n.back() - '0');
            auto fr = sw(strfmt("02:aa:00:00:00:0%d", k).c_str(),
                         strfmt("no-alert 10.20%d.0.%d/30", k, 4 * host[n] + 2).c_str());
            frames[n] = fr;
            if (carrier[n]) lldp_src->frames[n] = fr;
        };
        for (const auto& n : nics) {
            carrier[n] = true;
            host[n] = 1;
            describe(n);
        }
        uint64_t rng = seed;
        auto next = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
        int checked = 0, mismatches = 0, labelled_states = 0, readdressed = 0;
        std::string first_bad;
        a.on_monitor_tick = [&](int tick) {
            if (tick % 2 == 0) {
                bool want = std::all_of(nics.begin(), nics.end(), [&](const std::string& n) { return carrier[n]; });
                bool label = path_exists(f.cfg.labels.path());
                std::string bad;
                if (label != want) bad = strfmt("label %d, want %d", label, want);
                for (const auto& n : nics) {
                    if (!carrier[n]) continue;
                    const int k = int(n.back() - '0');
                    const std::string expect = strfmt("10.20%d.0.%d/30", k, 4 * host[n] + 1);
                    std::vector<std::string> have;
                    for (const auto& x : f.ops.addrs)
                        if (x.ifindex == idx[n]) have.push_back(x.prefix().str());
                    if (have != std::vector<std::string>{expect}) bad += " " + n + " holds " + join(have, ",") + " not " + expect;
                }
                ++checked;
                labelled_states += want;
                if (!bad.empty()) {
                    if (!mismatches) first_bad = strfmt("tick %d:", tick) + bad;
                    ++mismatches;
                }
                if (tick >= 400) stop.fire();
                return;
            }
            const std::string& n = nics[next() % nics.size()];
            if (next() % 3 == 0) {  // the switch port is re-addressed
                host[n] = 1 + int(next() % 8);
                ++readdressed;
                describe(n);
            } else {
                carrier[n] = !carrier[n];
                if (carrier[n])
                    lldp_src->frames[n] = frames[n];
                else
                    lldp_src->frames.erase(n);
                f.ops.set_carrier(n, carrier[n]);
            }
        };
        a.run(stop.fd[0]);
        if (mismatches) fprintf(stderr, "seed %llx, %d mismatches, first %s\n", (unsigned long long)seed, mismatches,
                                first_bad.c_str());
        CHECK_EQ(mismatches, 0);
        CHECK_EQ(checked, 201);
        CHECK(labelled_states > 0 && labelled_states < checked);
        CHECK(readdressed > 10);
    }
}

TEST(agent_firmware_lldp_records_of_nics_no_longer_selected_are_not_lost) {
    // The record an earlier agent left names ens0 (still selected), old0 (dropped from the
    // policy's interface list) and gone0 (renamed: unreachable).  old0 is not ours any more, so its
    // original goes back at once; gone0 cannot be reached and stays in the record for --cleanup,
    // also after this agent's own clean exit.
    for (bool keep : {true, false}) {
        Fixture f;
        f.cfg.keep_config = keep;
        f.cfg.disable_fw_lldp = true;
        f.cfg.lldp_cache = f.tmp.path + "/lldp-cache";
        f.cfg.fw_lldp_state = f.tmp.path + "/fw-lldp-state";
        write_file_atomic(f.cfg.fw_lldp_state, "ens0 priv 0x2\nold0 priv 0x4\ngone0 dcbx 0x0c\n");
        auto eth = std::make_unique<FakeEthtool>();
        eth->drivers = {{"ens0", "ice"}, {"old0", "ice"}};
        eth->flags["ens0"] = {{"link-down-on-close", "fw-lldp-agent"}, 0x0};  // already off (by the earlier agent)
        eth->flags["old0"] = {{"link-down-on-close", "fw-lldp-agent", "x"}, 0x0};
        FakeEthtool* raw = eth.get();
        Pipe stop;
        stop.fire();
        {
            agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
            a.set_ethtool_ops(std::move(eth));
            a.run(stop.fd[0]);
            CHECK(a.ready());
            CHECK_EQ(raw->flags["old0"].bits, uint32_t(0x4));  // restored at start
            // kept off across the restart / the true original back on the clean exit
            CHECK_EQ(raw->flags["ens0"].bits, uint32_t(keep ? 0x0 : 0x2));
        }
        auto st = read_file(f.cfg.fw_lldp_state);
        CHECK(st && *st == (keep ? "ens0 priv 0x2\ngone0 dcbx 0x0c\n" : "gone0 dcbx 0x0c\n"));
    }
}

TEST(agent_max_frame_boundaries_match_what_the_agent_advertises) {
    // One definition for sending and checking (802.3: header + payload + FCS, + 802.1Q tag on a
    // VLAN NIC): for MTU 9000, 9017 is refused and 9018 accepted; 1518 is enough for MTU 1500;
    // a tagged NIC needs 9022.
    CHECK_EQ(agent::max_frame_for_mtu(9000, false), 9018);
    CHECK_EQ(agent::max_frame_for_mtu(1500, false), 1518);
    CHECK_EQ(agent::max_frame_for_mtu(9000, true), 9022);
    struct Case {
        int mtu, frame;
        bool vlan, ok;
    };
    for (const Case c : {Case{9000, 9017, false, false}, Case{9000, 9018, false, true}, Case{1500, 1518, false, true},
                         Case{1500, 1517, false, false}, Case{9000, 9021, true, false}, Case{9000, 9022, true, true}}) {
        Fixture f;
        f.cfg.keep_running = false;
        f.cfg.mtu = c.mtu;
        f.cfg.interfaces = "ens1";
        if (c.vlan) f.ops.links["ens1"].kind = "vlan";
        auto src = f.all_valid();
        src->frames["ens1"].set_max_frame_size(uint16_t(c.frame));
        agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
        std::string err;
        try {
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        CHECK_EQ(err.empty(), c.ok);
        if (!c.ok)
            CHECK(err.find(strfmt("accepts frames up to %d bytes, but MTU %d needs %d%s", c.frame, c.mtu,
                                  agent::max_frame_for_mtu(c.mtu, c.vlan), c.vlan ? " (802.1Q tagged)" : "")) !=
                  std::string::npos);
    }
}

TEST(agent_invalid_rail_pattern_waits_with_one_reason_instead_of_crash_looping) {
    // A policy that reached the agent without admission (webhooks off) with a Python-only regex:
    // the agent touches nothing, says why in one line (status.json, the probe's reason file) and
    // waits for SIGTERM instead of exiting into a restart loop on every node.
    Fixture f;
    f.cfg.rail_switch_pattern = "(?i)leaf-r{rail}";
    f.tmp.write("features.d/scale-out-readiness.txt", "stale\n");
    Pipe stop;
    stop.fire();
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(stop.fd[0]);  // returns on the stop, no exception
    CHECK(!a.ready());
    CHECK(f.ops.addrs.empty());
    CHECK_EQ(f.ops.calls["link_set_up"], 0);
    CHECK(!path_exists(f.cfg.labels.path()));
    auto why = read_file(agent::reason_path(f.cfg.status_file));
    CHECK(why && why->find("invalid railSwitchPattern '(?i)leaf-r{rail}': ") == 0);
    CHECK(why->find("nothing configured") != std::string::npos);
    // One-shot runs (no --keep-running) and dry runs still fail fast.
    Fixture g;
    g.cfg.keep_running = false;
    g.cfg.rail_switch_pattern = "a{{rail},3}";  // fine for rails 0..3, a reversed range for rail 4
    agent::Agent b(g.cfg, g.ops, g.all_valid(), g.nm());
    std::string err;
    try {
        b.run(-1);
    } catch (const agent::AgentError& e) {
        err = e.what();
    }
    CHECK(err.find("(with {rail} = 4)") != std::string::npos);
    CHECK_EQ(agent::rail_pattern_error("leaf-r{rail}-.*"), std::string());
}

// ---------------------------------------------------------------------------------------------
// --require-rdma: the label (and rccl.env) wait for every NIC's RDMA device
// ---------------------------------------------------------------------------------------------
namespace {
struct RdmaFixture : Fixture {
    RdmaFixture() {
        cfg.require_rdma = true;
        cfg.sysfs_root = tmp.path + "/sys/";
        tmp.mkdir("sys/class/net");
        cfg.rccl_env = tmp.path + "/rccl.env";
        cfg.rdma_poll_ns = 1000000;
        cfg.monitor_tick_ns = 1000000;
        cfg.gid_wait_ns = 1000000;  // no GID tables in this sysfs
    }
    void bind(const std::string& nic, const std::string& dev) { tmp.mkdir("sys/class/net/" + nic + "/device/infiniband/" + dev); }
};
}  // namespace

TEST(agent_require_rdma_configures_waits_unlabelled_then_labels_when_the_devices_appear) {
    RdmaFixture f;
    f.tmp.write("rccl.env", "NCCL_IB_HCA==mlx5_9:1\n");  // an earlier run's, naming a device that is gone
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    bool waited = false, labelled = false;
    std::string reason;
    a.on_monitor_tick = [&](int tick) {
        if (tick == 1) {
            auto why = read_file(agent::reason_path(f.cfg.status_file));
            reason = why ? *why : "";
            waited = !path_exists(f.cfg.labels.path()) && !path_exists(f.cfg.rccl_env);
            for (int i = 0; i < 3; ++i) CHECK(a.nics()[size_t(i)].configured);  // the NICs are not held back
            f.bind("ens0", "mlx5_0");
            f.bind("ens1", "mlx5_1");
        } else if (tick == 20) {
            CHECK(!path_exists(f.cfg.labels.path()));  // ens2 still has none
            f.bind("ens2", "mlx5_2");
        } else if (tick > 20 && path_exists(f.cfg.labels.path())) {
            labelled = true;
            stop.fire();
        } else if (tick > 2000) {
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK(waited);
    CHECK_EQ(reason, std::string("ens0: waiting for RDMA device; ens1: waiting for RDMA device; ens2: waiting for RDMA device\n"));
    CHECK(labelled);
    auto env = read_file(f.cfg.rccl_env);
    CHECK(env && env->find("NCCL_IB_HCA==mlx5_0:1,mlx5_1:1,mlx5_2:1\n") != std::string::npos);
    CHECK(a.render_metrics().find("netop_agent_nic_rdma{nic=\"ens2\"} 1") != std::string::npos);
}

TEST(agent_require_rdma_devices_that_appear_during_the_bring_up_are_in_rccl_env_before_the_label) {
    // The RDMA driver finishes loading while the NICs are being configured: the artifacts were
    // written without the devices (rccl.env held back), the final check finds them all, and the
    // label must not be published over a missing rccl.env.
    RdmaFixture f;
    f.cfg.keep_running = true;
    bool bound = false;
    f.ops.on_op = [&](const std::string& op) {
        if (op == "addr_add" && !bound) {
            bound = true;
            f.bind("ens0", "mlx5_0");
            f.bind("ens1", "mlx5_1");
            f.bind("ens2", "mlx5_2");
        }
    };
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    bool labelled = false;
    std::optional<std::string> env;
    a.on_monitor_tick = [&](int) {  // the state the start left, before the monitor changes anything
        labelled = path_exists(f.cfg.labels.path());
        env = read_file(f.cfg.rccl_env);
        stop.fire();
    };
    a.run(stop.fd[0]);
    CHECK(bound);
    CHECK(labelled);
    CHECK(env && env->find("NCCL_IB_HCA==mlx5_0:1,mlx5_1:1,mlx5_2:1\n") != std::string::npos);
}

TEST(agent_label_and_rccl_env_follow_random_rdma_driver_reloads_and_flaps_in_l3_and_l2) {
    // Property (L3 and L2, --require-rdma, monitor): under any sequence of RDMA driver unloads, reloads
    // (which may number a device anew) and cable pulls, once the agent has caught up:
    //   the label is there exactly when every NIC has carrier and an RDMA device;
    //   while it is, rccl.env names exactly the current devices, in GPU order;
    //   while a device is missing, there is no rccl.env (no rail left to TCP sockets).
    // 120 random steps for each of three seeds.
    for (const char* mode : {"L3", "L2"})
    for (uint64_t seed : {0x0F1E2D3C4B5A6978ull, 0x1111222233334444ull, 0x9999AAAABBBBCCCCull}) {
        RdmaFixture f;
        f.cfg.mode = mode;
        f.cfg.xgmi_health_interval_ns = 1000000;  // a labelled node looks for its devices every 1 ms
        const std::vector<std::string> nics = {"ens0", "ens1", "ens2"};
        std::map<std::string, bool> carrier;
        std::map<std::string, std::string> dev;
        int next_dev = 0;
        for (const auto& n : nics) {
            carrier[n] = true;
            dev[n] = "mlx5_" + std::to_string(next_dev++);
            f.bind(n, dev[n]);
        }
        uint64_t rng = seed;
        auto next = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        int steps = 0, mismatches = 0, labelled_states = 0;
        int64_t t_step = 0;
        std::string first_bad;
        a.on_monitor_tick = [&](int) {
            if (t_step && mono_ns() - t_step < 20000000LL) return;  // 20 ms to catch up
            if (t_step) {  // check the state the last step led to
                const bool all_rdma = std::all_of(nics.begin(), nics.end(), [&](const std::string& n) { return !dev[n].empty(); });
                const bool want = all_rdma && std::all_of(nics.begin(), nics.end(), [&](const std::string& n) { return carrier[n]; });
                const bool label = path_exists(f.cfg.labels.path());
                auto env = read_file(f.cfg.rccl_env);
                std::string bad;
                if (label != want) bad = strfmt("label %d, want %d", label, want);
                if (!all_rdma && env) bad += " rccl.env while a device is missing";
                if (label) {
                    std::vector<std::string> hcas;
                    for (const auto& n : nics) hcas.push_back(dev[n] + ":1");
                    const std::string line = "NCCL_IB_HCA==" + join(hcas, ",") + "\n";
                    if (!env || env->find(line) == std::string::npos) bad += " rccl.env does not name " + join(hcas, ",");
                }
                if (!bad.empty() && mono_ns() - t_step < 2000000000LL) return;  // a loaded machine: up to 2 s more
                labelled_states += want;
                if (!bad.empty()) {
                    if (!mismatches) first_bad = strfmt("step %d:", steps) + bad;
                    ++mismatches;
                }
                if (++steps >= 120) {
                    stop.fire();
                    return;
                }
            }
            // Half the steps repair something broken (so the walk keeps coming back to a ready
            // node), the others break or repair at random.
            std::vector<std::string> broken;
            for (const auto& m : nics)
                if (!carrier[m] || dev[m].empty()) broken.push_back(m);
            const bool repair = !broken.empty() && next() % 2 == 0;
            const std::string& n = repair ? *std::find(nics.begin(), nics.end(), broken[next() % broken.size()])
                                          : nics[next() % nics.size()];
            if (repair ? !carrier[n] && (dev[n].size() || next() % 2) : next() % 3 == 0) {
                carrier[n] = !carrier[n];
                f.ops.set_carrier(n, carrier[n]);
            } else if (dev[n].empty()) {  // the driver loads again; a reload may renumber
                dev[n] = next() % 2 ? "mlx5_" + std::to_string(next_dev++) : "mlx5_" + std::to_string(&n - &nics[0]);
                bool taken = false;
                for (const auto& m : nics)
                    if (&m != &n && dev[m] == dev[n]) taken = true;
                if (taken) dev[n] = "mlx5_" + std::to_string(next_dev++);
                f.bind(n, dev[n]);
            } else {  // unloaded
                std::filesystem::remove_all(f.tmp.path + "/sys/class/net/" + n + "/device/infiniband");
                dev[n].clear();
            }
            t_step = mono_ns();
        };
        a.run(stop.fd[0]);
        if (mismatches) fprintf(stderr, "%s, seed %llx, %s\n", mode, (unsigned long long)seed, first_bad.c_str());
        CHECK_EQ(mismatches, 0);
        CHECK_EQ(steps, 120);
        if (labelled_states == 0 || labelled_states >= steps) fprintf(stderr, "seed %llx: %d labelled states\n", (unsigned long long)seed, labelled_states);
        CHECK(labelled_states > 0 && labelled_states < steps);  // the sequence visits both states
    }
}

TEST(agent_label_follows_random_pcie_retrains_and_cable_pulls_with_require_full_pcie) {
    // Property (L3 and L2, --require-full-pcie, monitor): under any sequence of a rail's PCIe link
    // retraining narrower (x8 of x16) or back to full width, and cable pulls, once the agent has
    // caught up the label is there exactly when every NIC has carrier and a full PCIe link.  The
    // monitor re-reads the links every 1 ms.  80 random steps for each of two seeds and modes.
    for (const char* mode : {"L3", "L2"})
    for (uint64_t seed : {0x5555AAAA5555AAAAull, 0x0123FEDC4567BA98ull}) {
        Fixture f;
        f.cfg.mode = mode;
        f.cfg.sysfs_root = f.tmp.path + "/sys/";
        f.cfg.require_full_pcie = true;
        f.cfg.xgmi_health_interval_ns = 1000000;
        f.cfg.monitor_tick_ns = 1000000;
        const std::vector<std::string> nics = {"ens0", "ens1", "ens2"};
        auto fn = [&](size_t k) { return strfmt("sys/devices/pci0000:00/0000:00:0%zu.0/0000:0%zu:00.0", k + 1, k + 1); };
        for (size_t k = 0; k < nics.size(); ++k) {
            const std::string port = strfmt("sys/devices/pci0000:00/0000:00:0%zu.0", k + 1);
            f.tmp.write(port + "/max_link_speed", "32.0 GT/s PCIe\n");
            f.tmp.write(port + "/max_link_width", "16\n");
            for (const char* a : {"max_link_speed", "current_link_speed"}) f.tmp.write(fn(k) + "/" + a, "32.0 GT/s PCIe\n");
            f.tmp.write(fn(k) + "/max_link_width", "16\n");
            f.tmp.write(fn(k) + "/current_link_width", "16\n");
            f.tmp.write(fn(k) + "/vendor", "0x15b3\n");
            f.tmp.mkdir("sys/class/net/" + nics[k]);
            f.tmp.mkdir("sys/bus/pci/devices");
            f.tmp.symlink(fn(k), "sys/class/net/" + nics[k] + "/device");
            f.tmp.symlink(fn(k), strfmt("sys/bus/pci/devices/0000:0%zu:00.0", k + 1));
        }
        std::map<std::string, bool> carrier, full;
        for (const auto& n : nics) carrier[n] = full[n] = true;
        uint64_t rng = seed;
        auto next = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        int steps = 0, mismatches = 0, labelled_states = 0;
        int64_t t_step = 0;
        std::string first_bad;
        a.on_monitor_tick = [&](int) {
            if (t_step && mono_ns() - t_step < 20000000LL) return;
            if (t_step) {
                const bool want = std::all_of(nics.begin(), nics.end(), [&](const std::string& n) { return carrier[n] && full[n]; });
                const bool label = path_exists(f.cfg.labels.path());
                if (label != want && mono_ns() - t_step < 2000000000LL) return;  // a loaded machine: up to 2 s more
                labelled_states += want;
                if (label != want) {
                    if (!mismatches) {
                        first_bad = strfmt("step %d: label %d, want %d;", steps, label, want);
                        for (const auto& n : nics) first_bad += strfmt(" %s carrier %d full %d", n.c_str(), carrier[n], full[n]);
                        first_bad += "\n" + read_file(f.cfg.status_file).value_or("");
                    }
                    ++mismatches;
                }
                if (++steps >= 80) {
                    stop.fire();
                    return;
                }
            }
            std::vector<size_t> broken;
            for (size_t k = 0; k < nics.size(); ++k)
                if (!carrier[nics[k]] || !full[nics[k]]) broken.push_back(k);
            const size_t k = !broken.empty() && next() % 2 ? broken[next() % broken.size()] : next() % nics.size();
            const std::string& n = nics[k];
            if ((!full[n] && (carrier[n] || next() % 2)) || (full[n] && carrier[n] && next() % 2)) {
                full[n] = !full[n];
                f.tmp.write(fn(k) + "/current_link_width", full[n] ? "16\n" : "8\n");
            } else {
                carrier[n] = !carrier[n];
                f.ops.set_carrier(n, carrier[n]);
            }
            t_step = mono_ns();
        };
        a.run(stop.fd[0]);
        if (mismatches) fprintf(stderr, "%s, seed %llx, %s\n", mode, (unsigned long long)seed, first_bad.c_str());
        CHECK_EQ(mismatches, 0);
        CHECK_EQ(steps, 80);
        CHECK(labelled_states > 0 && labelled_states < steps);
    }
}

TEST(agent_looks_up_the_gid_index_again_after_a_link_comes_back) {
    // The RDMA core drops a netdev's IP GIDs when the link goes down and adds them again when it
    // comes back, in whatever slot is free: ens1's RoCE v2 GID moves from index 3 to 5 during its
    // flap.  The republished rccl.env must not keep the stale NCCL_IB_GID_INDEX=3 (RCCL would use
    // another GID, or none, on that rail).
    RdmaFixture f;
    const std::map<std::string, std::string> ips = {{"ens0", "10.200.0.1"}, {"ens1", "10.200.0.5"}, {"ens2", "10.200.0.10"}};
    auto put_gid = [&](const std::string& dev, int idx, const std::string& ip, bool present) {
        const std::string d = "sys/class/infiniband/" + dev + "/ports/1/";
        auto ipv = *Ipv4::parse(ip);
        uint8_t b[4];
        ipv.to_net(b);
        f.tmp.write(d + "gids/" + std::to_string(idx),
                    present ? strfmt("0000:0000:0000:0000:0000:ffff:%02x%02x:%02x%02x\n", b[0], b[1], b[2], b[3])
                            : std::string("0000:0000:0000:0000:0000:0000:0000:0000\n"));
        f.tmp.write(d + "gid_attrs/types/" + std::to_string(idx), "RoCE v2\n");
    };
    for (int k = 0; k < 3; ++k) {
        const std::string nic = "ens" + std::to_string(k), dev = "mlx5_" + std::to_string(k);
        f.bind(nic, dev);
        put_gid(dev, 3, ips.at(nic), true);
    }
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    int phase = 0;
    std::string env_before, env_after;
    const int64_t t0 = mono_ns();
    a.on_monitor_tick = [&](int) {
        const bool labelled = path_exists(f.cfg.labels.path());
        if (phase == 0 && labelled) {
            env_before = read_file(f.cfg.rccl_env).value_or("");
            f.ops.set_carrier("ens1", false);
            phase = 1;
        } else if (phase == 1 && !labelled) {
            put_gid("mlx5_1", 3, ips.at("ens1"), false);  // gone with the link, back in another slot
            put_gid("mlx5_1", 5, ips.at("ens1"), true);
            f.ops.set_carrier("ens1", true);
            phase = 2;
        } else if (phase == 2 && labelled) {
            env_after = read_file(f.cfg.rccl_env).value_or("");
            phase = 3;
            stop.fire();
        } else if (mono_ns() - t0 > 5000000000LL) {
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK_EQ(phase, 3);
    CHECK(env_before.find("NCCL_IB_GID_INDEX=3\n") != std::string::npos);
    CHECK(env_after.find("NCCL_IB_GID_INDEX=3\n") == std::string::npos);  // not the stale index
    CHECK(env_after.find("NCCL_IB_ROCE_VERSION_NUM=2\n") != std::string::npos);  // 3 and 5: RCCL picks per HCA
    CHECK(env_after.find("NCCL_IB_HCA==mlx5_0:1,mlx5_1:1,mlx5_2:1\n") != std::string::npos);
}

TEST(agent_rccl_env_gid_index_is_never_stale_under_random_readdressing_and_flaps) {
    // Property (L3, RDMA on every rail, monitor): a simulated RDMA core keeps each device's RoCE v2
    // GID table -- an IPv4 GID appears in a free slot when the address is added, goes when it is
    // removed or its link goes down, and comes back (in whatever slot is free then) when the link
    // is up again.  Under random switch-port re-addressing and cable pulls, whenever the node is
    // labelled and rccl.env names NCCL_IB_GID_INDEX=k, slot k of every rail holds that rail's own
    // current address.  Three seeds, 100 steps each.
    for (uint64_t seed : {0x13579BDF2468ACE0ull, 0x0A0B0C0D0E0F1011ull, 0xFEEDFACECAFEF00Dull}) {
        RdmaFixture f;
        f.cfg.xgmi_health_interval_ns = 1000000;
        f.cfg.lldp_tx_interval_ns = 3600LL * 1000000000LL;
        f.cfg.gid_wait_ns = 50000000;  // the simulated core answers at once
        const std::vector<std::string> nics = {"ens0", "ens1", "ens2"};
        const std::map<int, std::string> by_index = {{10, "ens0"}, {11, "ens1"}, {12, "ens2"}};
        std::map<std::string, bool> carrier;
        std::map<std::string, int> host;
        std::map<std::string, std::map<int, uint32_t>> table;  // nic -> slot -> IPv4 (host order)
        uint64_t rng = seed;
        auto next = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        auto write_table = [&](const std::string& n) {
            const std::string dev = "mlx5_" + std::string(1, n.back());
            for (int slot = 0; slot < 8; ++slot) {
                const std::string d = "sys/class/infiniband/" + dev + "/ports/1/";
                auto it = table[n].find(slot);
                std::string gid = "0000:0000:0000:0000:0000:0000:0000:0000\n";
                if (it != table[n].end()) {
                    const uint32_t v = it->second;
                    gid = strfmt("0000:0000:0000:0000:0000:ffff:%04x:%04x\n", v >> 16, v & 0xffff);
                }
                f.tmp.write(d + "gids/" + std::to_string(slot), gid);
                f.tmp.write(d + "gid_attrs/types/" + std::to_string(slot), "RoCE v2\n");
            }
        };
        // The RDMA core: the GIDs follow each NIC's IPv4 addresses while its link is up.
        auto sync = [&] {
            for (const auto& n : nics) {
                std::set<uint32_t> want;
                if (carrier[n])
                    for (const auto& x : f.ops.addrs)
                        if (by_index.count(x.ifindex) && by_index.at(x.ifindex) == n && x.family == AF_INET) want.insert(x.local.v);
                auto& t = table[n];
                for (auto it = t.begin(); it != t.end();) it = want.count(it->second) ? std::next(it) : t.erase(it);
                for (uint32_t ip : want) {
                    bool have = false;
                    for (auto& [slot, v] : t) have |= v == ip;
                    if (have) continue;
                    // The lowest free slot half the time, a free slot from a random start otherwise.
                    for (int k = 0, start = next() % 2 ? 2 : 2 + int(next() % 6); k < 6; ++k) {
                        const int slot = 2 + (start - 2 + k) % 6;
                        if (!t.count(slot)) {
                            t[slot] = ip;
                            break;
                        }
                    }
                }
                write_table(n);
            }
        };
        f.ops.after_op = [&](const std::string&) { sync(); };
        auto src = f.all_valid();
        ScriptedLldp* lldp_src = src.get();
        std::map<std::string, lldp::Frame> frames;
        auto describe = [&](const std::string& n) {
            const int k = int(n.back() - '0');
            frames[n] = sw(strfmt("02:aa:00:00:00:0%d", k).c_str(), strfmt("no-alert 10.20%d.0.%d/30", k, 4 * host[n] + 2).c_str());
            if (carrier[n]) lldp_src->frames[n] = frames[n];
        };
        for (const auto& n : nics) {
            carrier[n] = true;
            host[n] = 1;
            describe(n);
            f.bind(n, "mlx5_" + std::string(1, n.back()));
            write_table(n);
        }
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, std::move(src), f.nm());
        int steps = 0, mismatches = 0, indexed = 0;
        int64_t t_step = 0;
        std::string first_bad;
        a.on_monitor_tick = [&](int) {
            if (t_step && mono_ns() - t_step < 20000000LL) return;
            if (t_step) {
                const bool want = std::all_of(nics.begin(), nics.end(), [&](const std::string& n) { return carrier[n]; });
                const bool label = path_exists(f.cfg.labels.path());
                std::string bad;
                if (label != want) bad = strfmt("label %d, want %d", label, want);
                auto env = read_file(f.cfg.rccl_env);
                if (label && env) {
                    const auto at = env->find("NCCL_IB_GID_INDEX=");
                    if (at != std::string::npos) {
                        const int k = std::atoi(env->c_str() + at + 18);
                        ++indexed;
                        for (const auto& n : nics) {
                            const int h = 4 * host[n] + 1, r = int(n.back() - '0');
                            const uint32_t ip = (10u << 24) | (uint32_t(200 + r) << 16) | uint32_t(h);
                            auto it = table[n].find(k);
                            if (it == table[n].end() || it->second != ip) bad += strfmt(" %s: slot %d is not its address", n.c_str(), k);
                        }
                    }
                }
                if (!bad.empty() && mono_ns() - t_step < 2000000000LL) return;
                if (!bad.empty()) {
                    if (!mismatches) first_bad = strfmt("step %d: ", steps) + bad;
                    ++mismatches;
                }
                if (++steps >= 100) {
                    stop.fire();
                    return;
                }
            }
            const std::string& n = nics[next() % nics.size()];
            if (carrier[n] && next() % 3 == 0) {  // the switch port is re-addressed
                host[n] = 1 + int(next() % 8);
                describe(n);
            } else {
                carrier[n] = !carrier[n];
                if (carrier[n])
                    lldp_src->frames[n] = frames[n];
                else
                    lldp_src->frames.erase(n);
                f.ops.set_carrier(n, carrier[n]);
                sync();  // the core drops / re-adds the link's GIDs
            }
            t_step = mono_ns();
        };
        a.run(stop.fd[0]);
        if (mismatches) fprintf(stderr, "seed %llx, %s\n", (unsigned long long)seed, first_bad.c_str());
        CHECK_EQ(mismatches, 0);
        CHECK_EQ(steps, 100);
        CHECK(indexed > 0);  // the walk did reach states with one index for every rail
    }
}

TEST(agent_monitor_never_blocks_on_a_gid_the_rdma_core_has_not_added_yet) {
    // After ens1's flap the RDMA core has not re-added its RoCE v2 GID yet.  The monitor
    // republishes the label at once (rccl.env without NCCL_IB_GID_INDEX: RCCL then picks each
    // HCA's RoCE v2 GID itself) instead of waiting out --gid-wait (2 s here) on its loop, and
    // names the index once the GID is there.
    RdmaFixture f;
    f.cfg.gid_wait_ns = 2000000000LL;
    const std::map<std::string, std::string> ips = {{"ens0", "10.200.0.1"}, {"ens1", "10.200.0.5"}, {"ens2", "10.200.0.10"}};
    auto put_gid = [&](const std::string& dev, const std::string& ip, bool present) {
        const std::string d = "sys/class/infiniband/" + dev + "/ports/1/";
        uint8_t b[4];
        Ipv4::parse(ip)->to_net(b);
        f.tmp.write(d + "gids/3", present ? strfmt("0000:0000:0000:0000:0000:ffff:%02x%02x:%02x%02x\n", b[0], b[1], b[2], b[3])
                                          : std::string("0000:0000:0000:0000:0000:0000:0000:0000\n"));
        f.tmp.write(d + "gid_attrs/types/3", "RoCE v2\n");
    };
    for (int k = 0; k < 3; ++k) {
        f.bind("ens" + std::to_string(k), "mlx5_" + std::to_string(k));
        put_gid("mlx5_" + std::to_string(k), ips.at("ens" + std::to_string(k)), true);
    }
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    int phase = 0;
    int64_t t_up = 0, t_gid = 0, up_to_label = -1, gid_to_env = -1;
    std::string env_without;
    const int64_t t0 = mono_ns();
    a.on_monitor_tick = [&](int) {
        const bool labelled = path_exists(f.cfg.labels.path());
        if (phase == 0 && labelled) {
            put_gid("mlx5_1", ips.at("ens1"), false);  // gone with the link
            f.ops.set_carrier("ens1", false);
            phase = 1;
        } else if (phase == 1 && !labelled) {
            f.ops.set_carrier("ens1", true);  // back, its GID not yet
            t_up = mono_ns();
            phase = 2;
        } else if (phase == 2 && labelled) {
            up_to_label = mono_ns() - t_up;
            env_without = read_file(f.cfg.rccl_env).value_or("");
            put_gid("mlx5_1", ips.at("ens1"), true);  // the core adds it now
            t_gid = mono_ns();
            phase = 3;
        } else if (phase == 3 && read_file(f.cfg.rccl_env).value_or("").find("NCCL_IB_GID_INDEX=3\n") != std::string::npos) {
            gid_to_env = mono_ns() - t_gid;
            phase = 4;
            stop.fire();
        } else if (mono_ns() - t0 > 8000000000LL) {
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK_EQ(phase, 4);
    CHECK(up_to_label >= 0 && up_to_label < 500000000LL);  // not the 2 s --gid-wait
    CHECK(env_without.find("NCCL_IB_GID_INDEX") == std::string::npos);
    CHECK(env_without.find("NCCL_IB_ROCE_VERSION_NUM=2\n") != std::string::npos);
    CHECK(gid_to_env >= 0 && gid_to_env < 1000000000LL);  // looked up again every 100 ms
    // rccl-net.json names each NIC's GID index too: rewritten with it (all three rails at 3)
    auto net = read_file(f.cfg.rccl_net).value_or("");
    size_t count = 0;
    for (size_t at = net.find("\"GID_INDEX\":3"); at != std::string::npos; at = net.find("\"GID_INDEX\":3", at + 1)) ++count;
    CHECK_EQ(count, size_t(3));
}

TEST(agent_require_rdma_past_the_wait_names_the_fault) {
    RdmaFixture f;
    f.cfg.rdma_wait_ns = 0;
    f.bind("ens1", "mlx5_1");
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    std::string reason;
    a.on_monitor_tick = [&](int tick) {
        if (tick == 2) {
            auto why = read_file(agent::reason_path(f.cfg.status_file));
            reason = why ? *why : "";
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK_EQ(reason, std::string("ens0: no RDMA device (load its RDMA driver); ens2: no RDMA device (load its RDMA driver)\n"));
    CHECK(!path_exists(f.cfg.labels.path()));
}

TEST(agent_require_rdma_without_the_monitor_fails_naming_the_nics) {
    RdmaFixture f;
    f.cfg.monitor = false;
    f.bind("ens0", "mlx5_0");
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    std::string err;
    try {
        a.run(-1);
    } catch (const agent::AgentError& e) {
        err = e.what();
    }
    CHECK(err.find("No RDMA device on ens1, ens2 (load the NIC's RDMA driver") == 0);
    CHECK(!path_exists(f.cfg.labels.path()));
}

TEST(agent_without_require_rdma_labels_nics_without_rdma_devices) {  // the reference's behaviour
    Fixture f;
    f.cfg.keep_running = false;
    f.cfg.rccl_env = f.tmp.path + "/rccl.env";
    f.cfg.gid_wait_ns = 1000000;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    auto env = read_file(f.cfg.rccl_env);
    CHECK(env && env->find("NCCL_IB_HCA") == std::string::npos);
}

// ---------------------------------------------------------------------------------------------
// --label-holddown: one withdrawal and one republish for a burst of flaps
// ---------------------------------------------------------------------------------------------
TEST(agent_label_holddown_republishes_once_after_the_last_flap) {
    Fixture f;
    f.cfg.monitor_tick_ns = 1000000;
    f.cfg.label_holddown_ns = 150LL * 1000000;
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    int withdrawals = 0, publishes = 0, flaps = 0;
    bool was = true;
    int64_t t_last_up = 0, t_back = 0, t_next = 0;
    std::string reason_in_holddown;
    a.on_monitor_tick = [&](int) {
        const bool now = path_exists(f.cfg.labels.path());
        if (was && !now) ++withdrawals;
        if (!was && now) {
            ++publishes;
            t_back = mono_ns();
        }
        was = now;
        auto& l = f.ops.links["ens1"];
        const int64_t t = mono_ns();
        if (flaps < 10 && t >= t_next) {  // ten flaps, 10 ms apart (down 5 ms, up 5 ms)
            const bool up = l.flags & IFF_UP;
            if (up) {
                l.flags &= ~unsigned(IFF_UP);
            } else {
                l.flags |= IFF_UP;
                ++flaps;
                t_last_up = t;
            }
            f.ops.events.push_back({false, l});
            t_next = t + 5000000;
        } else if (flaps == 10 && t_last_up && t - t_last_up > 20000000 && reason_in_holddown.empty()) {
            auto why = read_file(agent::reason_path(f.cfg.status_file));
            reason_in_holddown = why ? *why : "-";
        }
        if (publishes || (t_last_up && t - t_last_up > 2000000000LL)) stop.fire();
    };
    a.run(stop.fd[0]);
    CHECK_EQ(flaps, 10);
    CHECK_EQ(withdrawals, 1);
    CHECK_EQ(publishes, 1);
    CHECK(t_back - t_last_up >= f.cfg.label_holddown_ns);
    CHECK(t_back - t_last_up < f.cfg.label_holddown_ns + 100000000LL);
    CHECK(reason_in_holddown.rfind("label hold-down: healthy again after 1 withdrawal(s)", 0) == 0);
    CHECK(a.render_metrics().find("netop_agent_label_suppressed_total 9\n") != std::string::npos);
    CHECK(a.render_metrics().find("netop_agent_label_withdrawals_total 1\n") != std::string::npos);
}

TEST(agent_refuses_a_policy_routed_nic_that_holds_the_nodes_own_address) {
    // a NIC whose default route sits in a per-NIC policy-routing table is not the main
    // table's uplink -- but when it also holds the node's own address (the source its rule selects,
    // or any non-/30 the agent never installs) it is how the node reaches that network (a
    // source-routed management or storage NIC), and flushing it could cut the node off.  Refused,
    // naming the table and the address, unless --allow-policy-routed; a rail whose policy table
    // only serves a /30 of the agent's is configured.
    auto rule = [](uint32_t table, uint32_t prio, const char* src) {
        nl::RuleSpec r;
        r.table = table;
        r.priority = prio;
        if (src) {
            r.src = *Ipv4Prefix::parse(src);
            r.selective = true;
        }
        return r;
    };
    for (int variant : {0, 1, 2}) {
        Fixture f;
        f.cfg.mode = "L3";
        f.cfg.keep_running = false;
        f.cfg.allow_policy_routed = variant == 1;
        f.ops.rules = {rule(RT_TABLE_LOCAL, 0, nullptr), rule(101, 100, "192.168.1.0/24"),
                       rule(RT_TABLE_MAIN, 32766, nullptr), rule(RT_TABLE_DEFAULT, 32767, nullptr)};
        auto def = route(11, "0.0.0.0/0", "192.168.1.1", RTPROT_STATIC);
        def.table = 101;
        f.ops.routes.push_back(def);
        // variant 2: the agent's own /30 from an earlier run (not in the rule's source)
        f.ops.addr_add(11, *Ipv4Prefix::parse(variant == 2 ? "10.200.0.5/30" : "192.168.1.5/24"));
        std::string err;
        try {
            agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
            a.run(-1);
        } catch (const agent::AgentError& e) {
            err = e.what();
        }
        if (variant == 0) {
            CHECK(err.find("Refusing to configure ens1 (a default route in policy-routing table 101 and the node's address "
                           "192.168.1.5/24, the source its rule 'from 192.168.1.0/24 lookup 101' selects): the node "
                           "reaches a network through it") == 0);
            CHECK(err.find("--allow-policy-routed") != std::string::npos);
            CHECK_EQ(f.ops.calls["link_set_up"], 0);
            CHECK_EQ(f.ops.addrs.size(), size_t(1));  // its address untouched
        } else {
            CHECK_EQ(err, std::string());
            CHECK_EQ(f.ops.addrs.size(), size_t(3));  // every NIC configured, ens1 too
        }
    }
    // A dry run names it as refused.
    Fixture f;
    f.cfg.mode = "L3";
    f.cfg.dry_run = true;
    f.ops.rules = {rule(101, 100, "192.168.1.0/24"), rule(RT_TABLE_MAIN, 32766, nullptr)};
    auto def = route(11, "0.0.0.0/0", "192.168.1.1", RTPROT_STATIC);
    def.table = 101;
    f.ops.routes.push_back(def);
    f.ops.addr_add(11, *Ipv4Prefix::parse("172.16.9.3/16"));  // not the rule's source, but no /30 either
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    a.run(-1);
    CHECK_EQ(a.excluded().size(), size_t(1));
    CHECK_EQ(a.excluded()[0].second, std::string("carries a default route in policy-routing table 101 and the node's "
                                                 "address 172.16.9.3/16, an address the agent never installs (not a "
                                                 "/30) (refused)"));
}

// ---------------------------------------------------------------------------------------------
// The monitor's gpu_metrics reads run on a worker; a link counts as down only on
// --xgmi-down-samples consecutive samples.
// ---------------------------------------------------------------------------------------------
namespace {
void write_two_gpu_kfd(const TmpDir& t) {
    const std::string base = "sys/class/kfd/kfd/topology/nodes/";
    t.write(base + "0/properties", "cpu_cores_count 96\nsimd_count 0\n");
    for (int g = 1; g <= 2; ++g) {
        t.write(base + std::to_string(g) + "/properties",
                strfmt("simd_count 1024\nvendor_id 4098\ndevice_id 30115\nlocation_id %d\ndomain 0\nhive_id 77\n", (g * 0x10) << 8));
        t.write(base + std::to_string(g) + "/io_links/0/properties",
                strfmt("type 11\nnode_from %d\nnode_to %d\nweight 15\nmin_bandwidth 76000\nmax_bandwidth 76000\n", g, 3 - g));
    }
    auto blob = read_file(std::string(NETOP_TEST_FIXTURES) + "/gpu_metrics_v1_8.bin");
    for (const char* bdf : {"0000:10:00.0", "0000:20:00.0"}) t.write(std::string("sys/bus/pci/devices/") + bdf + "/gpu_metrics", *blob);
}

void set_link(const TmpDir& t, const char* bdf, int slot, bool up) {
    const std::string path = t.path + "/sys/bus/pci/devices/" + bdf + "/gpu_metrics";
    std::string b = *read_file(path);
    b[264 + 2 * size_t(slot)] = up ? 1 : 0;
    b[265 + 2 * size_t(slot)] = 0;
    write_file_atomic(path, b);
}
}  // namespace

TEST(agent_monitor_reads_gpu_metrics_on_a_worker_and_dampens_a_single_down_sample) {
    for (int samples : {2, 1000000}) {
        Fixture f;
        f.cfg.sysfs_root = f.tmp.path + "/sys/";
        f.cfg.xgmi_expect_links = 0;
        f.cfg.xgmi_health_interval_ns = 2000000;  // 2 ms
        f.cfg.xgmi_down_samples = samples;
        f.cfg.monitor_tick_ns = 1000000;
        write_two_gpu_kfd(f.tmp);
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        int64_t t_down = 0;
        bool withdrawn = false, back = false;
        std::string reason;
        a.on_monitor_tick = [&](int tick) {
            if (tick == 1) {
                CHECK(path_exists(f.cfg.labels.path()));
                set_link(f.tmp, "0000:20:00.0", 3, false);
                t_down = mono_ns();
            } else if (t_down && !withdrawn && !path_exists(f.cfg.labels.path())) {
                withdrawn = true;
                auto why = read_file(agent::reason_path(f.cfg.status_file));
                reason = why ? *why : "";
                set_link(f.tmp, "0000:20:00.0", 3, true);
            } else if (withdrawn && path_exists(f.cfg.labels.path())) {
                back = true;
                stop.fire();
            } else if (t_down && mono_ns() - t_down > 300000000LL) {
                stop.fire();  // 300 ms: ~150 samples
            }
        };
        a.run(stop.fd[0]);
        if (samples == 2) {
            CHECK(withdrawn && back);
            CHECK_EQ(reason, std::string("xGMI: GPU 0000:20:00.0: link 3 down\n"));
        } else {
            CHECK(!withdrawn);  // never enough consecutive samples
        }
    }
}

namespace {
size_t count_dir(const std::string& dir) {
    size_t n = 0;
    for (const auto& e : std::filesystem::directory_iterator(dir)) (void)e, ++n;
    return n;
}
}  // namespace

TEST(agent_monitor_health_worker_soak_leaves_no_threads_or_descriptors_behind) {
    // The monitor's xGMI / PCIe poll runs on detached workers per sample, signalled through an
    // eventfd: a poll every millisecond for a second is a thousand samples.  Once the agent is
    // gone, so are its threads and descriptors, and the monitor still acted on a link that went
    // down after the soak.
    const size_t threads_before = count_dir("/proc/self/task"), fds_before = count_dir("/proc/self/fd");
    bool withdrawn = false;
    {
        Fixture f;
        f.cfg.sysfs_root = f.tmp.path + "/sys/";
        f.cfg.xgmi_expect_links = 0;
        f.cfg.xgmi_health_interval_ns = 1000000;  // 1 ms
        f.cfg.require_full_pcie = true;           // the PCIe half of the sample too
        f.cfg.monitor_tick_ns = 1000000;
        write_two_gpu_kfd(f.tmp);
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        int64_t t_base = 0, t_down = 0;
        a.on_monitor_tick = [&](int tick) {
            if (tick == 1) {
                t_base = mono_ns();
            } else if (t_base && !t_down && mono_ns() - t_base > 1000000000LL) {
                set_link(f.tmp, "0000:10:00.0", 2, false);
                t_down = mono_ns();
            } else if (t_down && !path_exists(f.cfg.labels.path())) {
                withdrawn = true;
                stop.fire();
            } else if (t_down && mono_ns() - t_down > 3000000000LL) {
                stop.fire();
            }
        };
        a.run(stop.fd[0]);
        CHECK(a.render_metrics().find("netop_agent_sysfs_reads_late_total{read=\"gpu_metrics\"} 0\n") != std::string::npos);
    }
    CHECK(withdrawn);
    // Detached workers finish on their own: give the last ones a moment.
    const int64_t until = mono_ns() + 3000000000LL;
    while ((count_dir("/proc/self/task") > threads_before || count_dir("/proc/self/fd") > fds_before) && mono_ns() < until)
        ::usleep(5000);
    CHECK(count_dir("/proc/self/task") <= threads_before);
    CHECK(count_dir("/proc/self/fd") <= fds_before);
}

TEST(agent_counts_sysfs_reads_that_miss_the_deadline) {
    // GPU 0000:20:00.0's gpu_metrics never answers (a FIFO nobody writes, as a wedged SMU): every
    // sample counts it late, by what was read, in netop_agent_sysfs_reads_late_total.
    Fixture f;
    f.cfg.sysfs_root = f.tmp.path + "/sys/";
    f.cfg.xgmi_expect_links = 0;
    f.cfg.xgmi_health_interval_ns = 2000000;
    f.cfg.sysfs_read_timeout_ns = 20000000;  // 20 ms
    f.cfg.monitor_tick_ns = 1000000;
    write_two_gpu_kfd(f.tmp);
    const std::string fifo = f.tmp.path + "/sys/bus/pci/devices/0000:20:00.0/gpu_metrics";
    ::unlink(fifo.c_str());
    CHECK_EQ(::mkfifo(fifo.c_str(), 0600), 0);
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    std::string metrics;
    const int64_t t0 = mono_ns();
    a.on_monitor_tick = [&](int) {
        metrics = a.render_metrics();
        if (metrics.find("netop_agent_sysfs_reads_late_total{read=\"gpu_metrics\"} 3\n") != std::string::npos ||
            mono_ns() - t0 > 3000000000LL)
            stop.fire();
    };
    a.run(stop.fd[0]);
    int w = ::open(fifo.c_str(), O_WRONLY | O_NONBLOCK | O_CLOEXEC);  // let the blocked reader go
    if (w >= 0) ::close(w);
    CHECK(metrics.find("netop_agent_sysfs_reads_late_total{read=\"gpu_metrics\"} 3\n") != std::string::npos);
    CHECK(metrics.find("netop_agent_sysfs_reads_late_total{read=\"pcie\"} 0\n") != std::string::npos);
    CHECK(!path_exists(f.cfg.labels.path()));  // a GPU whose links cannot be read is not labelled
}

TEST(agent_label_holddown_and_xgmi_dampening_follow_random_link_and_carrier_flaps) {
    // Property (L3, monitor, --label-holddown 100 ms, --xgmi-down-samples 2): under any sequence
    // of cable pulls and xGMI links going down / up, checked 10 ms or 150 ms after each step:
    //   unhealthy (a NIC without carrier or a GPU link down): no label;
    //   healthy and never withdrawn: the label (the first publication is not held);
    //   healthy after a withdrawal: the label only once the hold-down has passed since the last
    //   change (so not at 10 ms, and at 150 ms).
    // 60 random steps for each of two seeds.
    for (uint64_t seed : {0x2468ACE013579BDFull, 0x0DDBA11C0FFEE000ull}) {
        Fixture f;
        f.cfg.sysfs_root = f.tmp.path + "/sys/";
        f.cfg.xgmi_expect_links = 0;
        f.cfg.xgmi_health_interval_ns = 1000000;
        f.cfg.xgmi_down_samples = 2;
        f.cfg.label_holddown_ns = 100000000;  // 100 ms
        f.cfg.monitor_tick_ns = 1000000;
        write_two_gpu_kfd(f.tmp);
        const std::vector<std::string> nics = {"ens0", "ens1", "ens2"};
        const std::vector<const char*> gpus = {"0000:10:00.0", "0000:20:00.0"};
        std::map<std::string, bool> carrier, link;
        for (const auto& n : nics) carrier[n] = true;
        for (const char* g : gpus) link[g] = true;
        uint64_t rng = seed;
        auto next = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        auto healthy = [&] {
            return std::all_of(nics.begin(), nics.end(), [&](const std::string& n) { return carrier[n]; }) &&
                   std::all_of(gpus.begin(), gpus.end(), [&](const char* g) { return link[g]; });
        };
        Pipe stop;
        agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
        bool labelled = true;  // the model: the start labels a healthy node
        int withdrawals = 0, steps = 0, mismatches = 0, held = 0;
        int64_t t_step = 0, wait = 0;
        std::string first_bad;
        a.on_monitor_tick = [&](int) {
            if (t_step && mono_ns() - t_step < wait) return;
            if (t_step) {
                bool want;
                if (!healthy())
                    want = false;
                else if (labelled || withdrawals == 0)
                    want = true;
                else
                    want = wait > f.cfg.label_holddown_ns;  // healthy since this step
                const bool label = path_exists(f.cfg.labels.path());
                // A held label is checked at once (the agent's hold-down starts when it sees the
                // health, after the step, so lateness can only keep it off longer).  Every other
                // expectation is a state the agent converges to: on a loaded machine it gets up to
                // 2 s more to reach it.
                const bool holding = healthy() && !want;
                if (label != want && !holding && mono_ns() - t_step < wait + 2000000000LL) return;
                // An unhealthy node: the agent must have seen it before the next step (an xGMI link
                // down for less than two samples is no flap, by design; on a loaded machine 10 ms
                // may hold one sample).  Its reason names the fault, not the hold-down.
                if (!healthy() && mono_ns() - t_step < wait + 2000000000LL) {
                    auto why = read_file(agent::reason_path(f.cfg.status_file));
                    if (!why || why->find("label hold-down") != std::string::npos) return;
                }
                held += holding;
                if (want) labelled = true;
                if (label != want) {
                    if (!mismatches)
                        first_bad = strfmt("step %d (waited %lld ms, %d withdrawal(s)): label %d, want %d", steps,
                                           (long long)(wait / 1000000), withdrawals, label, want);
                    ++mismatches;
                }
                if (++steps >= 60) {
                    stop.fire();
                    return;
                }
            }
            // A balanced walk: half the steps repair something broken.
            std::vector<int> broken;  // 0..2 NICs, 3..4 GPUs
            for (int i = 0; i < 3; ++i)
                if (!carrier[nics[size_t(i)]]) broken.push_back(i);
            for (int i = 0; i < 2; ++i)
                if (!link[gpus[size_t(i)]]) broken.push_back(3 + i);
            const int what = !broken.empty() && next() % 2 ? broken[next() % broken.size()] : int(next() % 5);
            if (what < 3) {
                const std::string& n = nics[size_t(what)];
                carrier[n] = !carrier[n];
                f.ops.set_carrier(n, carrier[n]);
            } else {
                const char* g = gpus[size_t(what - 3)];
                link[g] = !link[g];
                set_link(f.tmp, g, 3, link[g]);
            }
            if (!healthy() && labelled) {
                labelled = false;
                ++withdrawals;
            }
            wait = next() % 2 ? 10000000LL : 150000000LL;
            t_step = mono_ns();
        };
        a.run(stop.fd[0]);
        if (mismatches) fprintf(stderr, "seed %llx, %s\n", (unsigned long long)seed, first_bad.c_str());
        CHECK_EQ(mismatches, 0);
        CHECK_EQ(steps, 60);
        CHECK(withdrawals > 0 && held > 0);  // the walk withdrew the label and held it back
    }
}

TEST(agent_require_rdma_withdraws_the_label_when_a_device_goes_away_and_follows_a_renumbered_one) {
    // After readiness the RDMA driver is unloaded under a labelled node: the label goes at the
    // next look (the health interval), with a fault reason (not start-up); the driver is loaded
    // again and numbers the device anew: the label comes back and rccl.env names the new HCA.
    RdmaFixture f;
    f.cfg.xgmi_health_interval_ns = 5000000;  // how often a labelled node looks again
    f.bind("ens0", "mlx5_0");
    f.bind("ens1", "mlx5_1");
    f.bind("ens2", "mlx5_2");
    Pipe stop;
    agent::Agent a(f.cfg, f.ops, f.all_valid(), f.nm());
    int phase = 0;
    std::string reason;
    int64_t t_unload = 0;
    bool env_while_gone = true;
    a.on_monitor_tick = [&](int tick) {
        const bool labelled = path_exists(f.cfg.labels.path());
        if (phase == 0 && labelled) {
            std::filesystem::remove_all(f.tmp.path + "/sys/class/net/ens1/device/infiniband");
            t_unload = mono_ns();
            phase = 1;
        } else if (phase == 1 && !labelled) {
            auto why = read_file(agent::reason_path(f.cfg.status_file));
            reason = why ? *why : "";
            env_while_gone = path_exists(f.cfg.rccl_env);
            f.bind("ens1", "mlx5_7");
            phase = 2;
        } else if (phase == 2 && labelled) {
            phase = 3;
            stop.fire();
        } else if (tick > 5000 || (t_unload && mono_ns() - t_unload > 2000000000LL)) {
            stop.fire();
        }
    };
    a.run(stop.fd[0]);
    CHECK_EQ(phase, 3);
    CHECK_EQ(reason, std::string("ens1: no RDMA device (load its RDMA driver)\n"));
    CHECK(!env_while_gone);  // no rccl.env naming mlx5_1 while it is gone
    auto env = read_file(f.cfg.rccl_env);
    CHECK(env && env->find("NCCL_IB_HCA==mlx5_0:1,mlx5_7:1,mlx5_2:1\n") != std::string::npos);
}
