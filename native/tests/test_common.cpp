#include "check.hpp"
#include "netop/cli.hpp"
#include "netop/common.hpp"

using namespace netop;

TEST(mac_parse_and_format) {
    auto m = MacAddr::parse("AA:bb:0c:dd:ee:0F");
    CHECK(m);
    CHECK_EQ(m->str(), std::string("aa:bb:0c:dd:ee:0f"));
    CHECK(!MacAddr::parse("aa:bb:cc:dd:ee"));
    CHECK(!MacAddr::parse("aa:bb:cc:dd:ee:gg"));
    CHECK(MacAddr::parse("00-11-22-33-44-55"));
}

TEST(ipv4_parse_strict) {
    CHECK_EQ(Ipv4::parse("10.200.10.2")->str(), std::string("10.200.10.2"));
    CHECK(!Ipv4::parse("10.200.10"));
    CHECK(!Ipv4::parse("10.200.10.256"));
    CHECK(!Ipv4::parse("10.200.010.2"));  // leading zero rejected like Go
    CHECK(!Ipv4::parse("10.200.10.2 "));
    CHECK(!Ipv4::parse(""));
}

TEST(prefix_parse_and_mask) {
    auto p = Ipv4Prefix::parse("10.200.10.2/30");
    CHECK(p);
    CHECK_EQ(p->len, 30);
    CHECK_EQ(p->network().str(), std::string("10.200.10.0"));
    CHECK_EQ(p->mask().str(), std::string("255.255.255.252"));
    CHECK(!Ipv4Prefix::parse("10.0.0.1/33"));
    CHECK(!Ipv4Prefix::parse("10.0.0.1/"));
    CHECK(!Ipv4Prefix::parse("10.0.0.1/030"));
    CHECK(!Ipv4Prefix::parse("10.0.0.1"));
    CHECK_EQ(Ipv4Prefix::parse("10.200.10.1/16")->masked().str(), std::string("10.200.0.0/16"));
}

TEST(split_semantics_match_go) {
    auto v = split("a  b", ' ');
    CHECK_EQ(v.size(), size_t(3));
    CHECK_EQ(v[1], std::string(""));
    CHECK_EQ(split("", ' ').size(), size_t(1));
    auto f = split_ws("  a \t b  ");
    CHECK_EQ(f.size(), size_t(2));
    CHECK_EQ(f[1], std::string("b"));
}

TEST(go_durations) {
    CHECK_EQ(*parse_go_duration("90s"), int64_t(90) * 1000000000);
    CHECK_EQ(*parse_go_duration("1m30s"), int64_t(90) * 1000000000);
    CHECK_EQ(*parse_go_duration("250ms"), int64_t(250) * 1000000);
    CHECK_EQ(*parse_go_duration("1.5s"), int64_t(1500) * 1000000);
    CHECK_EQ(*parse_go_duration("0"), int64_t(0));
    CHECK_EQ(*parse_go_duration("2h"), int64_t(7200) * 1000000000);
    CHECK(!parse_go_duration("90"));
    CHECK(!parse_go_duration("s"));
    CHECK(!parse_go_duration("5x"));
    CHECK_EQ(format_go_duration(int64_t(90) * 1000000000), std::string("1m30s"));
    CHECK_EQ(format_go_duration(int64_t(30) * 1000000000), std::string("30s"));
}

TEST(flagset_pflag_semantics) {
    std::string mode = "L3", ifaces;
    bool configure = false, keep = false;
    int mtu = 1500, v = 0;
    int64_t wait = 30000000000LL;
    cli::FlagSet fs("discover");
    fs.add_string("mode", &mode, "");
    fs.add_bool("configure", &configure, "");
    fs.add_bool("keep-running", &keep, "");
    fs.add_string("interfaces", &ifaces, "");
    fs.add_int("mtu", &mtu, "");
    fs.add_int("v", &v, "");
    fs.shorthand('v', "v");
    fs.add_duration("wait", &wait, "");
    fs.alias("gaudinet", "interfaces");
    const char* argv[] = {"discover", "--configure=true", "--keep-running", "--mode", "l2", "--mtu=9000",
                          "-v", "3", "--wait=90s", "--gaudinet=x"};
    fs.parse(10, const_cast<char**>(argv));
    CHECK(configure);
    CHECK(keep);
    CHECK_EQ(mode, std::string("l2"));
    CHECK_EQ(mtu, 9000);
    CHECK_EQ(v, 3);
    CHECK_EQ(wait, int64_t(90) * 1000000000);
    CHECK_EQ(ifaces, std::string("x"));
    const char* bad[] = {"discover", "--nope"};
    CHECK_THROWS(fs.parse(2, const_cast<char**>(bad)));
    const char* badbool[] = {"discover", "--configure=maybe"};
    CHECK_THROWS(fs.parse(2, const_cast<char**>(badbool)));
    const char* baddur[] = {"discover", "--wait=90"};
    CHECK_THROWS(fs.parse(2, const_cast<char**>(baddur)));
}

#include <linux/netlink.h>
#include <linux/rtnetlink.h>
#include <sys/socket.h>

#include <cstring>

#include "netop/netlink.hpp"

TEST(netlink_parse_link_rejects_truncated_and_unaligned_input) {
    // Regressions found by the netlink fuzz target (make fuzz-native).
    std::vector<uint8_t> buf(NLMSG_HDRLEN + 4, 0);
    auto* h = reinterpret_cast<nlmsghdr*>(buf.data());
    h->nlmsg_len = uint32_t(buf.size());  // shorter than nlmsghdr + ifinfomsg
    h->nlmsg_type = RTM_NEWLINK;
    CHECK_THROWS(netop::nl::parse_link(h));
    // ifinfomsg + one IFLA_IFNAME attribute whose unaligned length ends the message exactly:
    // RTA_NEXT's aligned step is larger than what is left and must not wrap the length.
    std::vector<uint8_t> m(NLMSG_LENGTH(sizeof(ifinfomsg)) + 5, 0);
    auto* h2 = reinterpret_cast<nlmsghdr*>(m.data());
    h2->nlmsg_len = uint32_t(m.size());
    h2->nlmsg_type = RTM_NEWLINK;
    auto* a = reinterpret_cast<rtattr*>(m.data() + NLMSG_LENGTH(sizeof(ifinfomsg)));
    a->rta_len = 5;
    a->rta_type = IFLA_IFNAME;
    m.back() = 'x';
    auto li = netop::nl::parse_link(h2);
    CHECK_EQ(li.name, std::string("x"));
}

TEST(netlink_parse_route_reads_multipath_next_hops_and_bounds_them) {
    // A default route over two next hops (ifindex 3 and 7): both are uplinks.  Then the same with
    // the second next hop's length claiming more than the attribute holds: only the first counts.
    auto build = [](uint16_t second_len) {
        std::vector<uint8_t> m(NLMSG_LENGTH(sizeof(rtmsg)), 0);
        auto put_hop = [&](std::vector<uint8_t>& v, int ifindex, uint16_t len) {
            rtnexthop nh{};
            nh.rtnh_len = len;
            nh.rtnh_ifindex = ifindex;
            const size_t off = v.size();
            v.resize(off + RTNH_ALIGN(sizeof nh), 0);
            std::memcpy(v.data() + off, &nh, sizeof nh);
        };
        std::vector<uint8_t> hops;
        put_hop(hops, 3, sizeof(rtnexthop));
        put_hop(hops, 7, second_len);
        const size_t aoff = m.size();
        m.resize(aoff + RTA_LENGTH(hops.size()), 0);
        auto* a = reinterpret_cast<rtattr*>(m.data() + aoff);
        a->rta_type = RTA_MULTIPATH;
        a->rta_len = uint16_t(RTA_LENGTH(hops.size()));
        std::memcpy(RTA_DATA(a), hops.data(), hops.size());
        auto* h = reinterpret_cast<nlmsghdr*>(m.data());
        h->nlmsg_len = uint32_t(m.size());
        h->nlmsg_type = RTM_NEWROUTE;
        auto* rt = reinterpret_cast<rtmsg*>(NLMSG_DATA(h));
        rt->rtm_family = AF_INET;
        rt->rtm_table = RT_TABLE_MAIN;
        rt->rtm_type = RTN_UNICAST;
        rt->rtm_dst_len = 0;
        return m;
    };
    auto ok = build(sizeof(rtnexthop));
    auto r = netop::nl::parse_route(reinterpret_cast<nlmsghdr*>(ok.data()));
    CHECK_EQ(r.dst.len, 0);
    CHECK_EQ(r.nexthops.size(), size_t(2));
    CHECK(r.nexthops == std::vector<int>({3, 7}));
    auto bad = build(200);  // longer than what is left of the attribute
    auto r2 = netop::nl::parse_route(reinterpret_cast<nlmsghdr*>(bad.data()));
    CHECK(r2.nexthops == std::vector<int>({3}));
}

TEST(netlink_parse_rule_tells_selective_rules_from_lookup_everything) {
    // `from all lookup main` selects nothing; a source prefix, an input interface or a non-zero
    // fwmark make a rule selective (per-NIC policy routing); FRA_TABLE overrides the header's
    // table (ids above 255); a truncated message is no rule.
    struct Hdr {
        uint8_t family, dst_len, src_len, tos, table, res1, res2, action;
        uint32_t flags;
    };
    auto build = [](uint8_t src_len, std::vector<std::pair<uint16_t, std::vector<uint8_t>>> attrs) {
        std::vector<uint8_t> m(NLMSG_LENGTH(sizeof(Hdr)), 0);
        for (auto& [type, payload] : attrs) {
            const size_t off = m.size();
            m.resize(off + RTA_SPACE(payload.size()), 0);
            auto* a = reinterpret_cast<rtattr*>(m.data() + off);
            a->rta_type = type;
            a->rta_len = uint16_t(RTA_LENGTH(payload.size()));
            std::memcpy(RTA_DATA(a), payload.data(), payload.size());
        }
        auto* h = reinterpret_cast<nlmsghdr*>(m.data());
        h->nlmsg_len = uint32_t(m.size());
        h->nlmsg_type = RTM_NEWRULE;
        auto* f = reinterpret_cast<Hdr*>(NLMSG_DATA(h));
        f->family = AF_INET;
        f->src_len = src_len;
        f->table = RT_TABLE_MAIN;
        f->action = 1;
        return m;
    };
    auto u32 = [](uint32_t v) {
        std::vector<uint8_t> b(4);
        std::memcpy(b.data(), &v, 4);
        return b;
    };
    auto parse = [](std::vector<uint8_t>& m) { return netop::nl::parse_rule(reinterpret_cast<nlmsghdr*>(m.data())); };
    auto all = build(0, {{6, u32(32766)}});  // FRA_PRIORITY
    auto r = parse(all);
    CHECK(r && !r->selective && r->table == RT_TABLE_MAIN && r->priority == 32766 && r->action == 1);
    auto from = build(24, {{2, {192, 168, 50, 0}}, {15, u32(1001)}});  // FRA_SRC, FRA_TABLE
    r = parse(from);
    CHECK(r && r->selective && r->table == 1001u && r->src.str() == "192.168.50.0/24");
    auto iif = build(0, {{3, {'e', 't', 'h', '0', 0}}});  // FRA_IIFNAME
    CHECK(parse(iif)->selective);
    auto mark0 = build(0, {{10, u32(0)}});  // FRA_FWMARK 0: matches every packet
    CHECK(!parse(mark0)->selective);
    auto mark = build(0, {{10, u32(7)}});
    CHECK(parse(mark)->selective);
    std::vector<uint8_t> shortmsg(NLMSG_LENGTH(4), 0);
    reinterpret_cast<nlmsghdr*>(shortmsg.data())->nlmsg_len = uint32_t(shortmsg.size());
    CHECK(!parse(shortmsg));
}

// ---------------------------------------------------------------------------------------------
// bounded.hpp: reads that may never return (a wedged SMU behind gpu_metrics), waited for with a
// deadline; a read still blocked is joined, never started twice.
// ---------------------------------------------------------------------------------------------
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "netop/bounded.hpp"
#include "tmpdir.hpp"

TEST(bounded_reads_return_at_the_deadline_and_join_a_read_still_blocked) {
    TmpDir t;
    t.write("plain", "1.8 metrics");
    const std::string fifo = t.path + "/stalled";
    CHECK_EQ(::mkfifo(fifo.c_str(), 0600), 0);
    const size_t before = bounded::in_flight();
    int64_t t0 = mono_ns();
    auto r = bounded::read_files({t.path + "/plain", fifo, t.path + "/missing"}, mono_ns() + 100000000LL);
    const int64_t took = mono_ns() - t0;
    CHECK(took >= 90000000LL && took < 1000000000LL);  // the deadline, not the stalled read
    CHECK(r[0].data && *r[0].data == "1.8 metrics" && !r[0].late);
    CHECK(!r[1].data && r[1].late);
    CHECK(!r[2].data && !r[2].late);  // unreadable is not late
    CHECK_EQ(bounded::in_flight(), before + 1);
    // Asked again while still blocked: joined (no second thread), late again.
    auto again = bounded::read_files({fifo}, mono_ns() + 20000000LL);
    CHECK(again[0].late);
    CHECK_EQ(bounded::in_flight(), before + 1);
    // The "SMU" answers: the blocked read returns its data, and the next read starts afresh.
    int w = ::open(fifo.c_str(), O_WRONLY | O_NONBLOCK);
    CHECK(w >= 0);
    CHECK_EQ(::write(w, "late answer", 11), 11);
    ::close(w);
    for (int i = 0; i < 200 && bounded::in_flight() > before; ++i) ::usleep(1000);
    CHECK_EQ(bounded::in_flight(), before);
    ::unlink(fifo.c_str());
    t.write("stalled", "fresh");
    auto fresh = bounded::read_files({fifo}, mono_ns() + 100000000LL);
    CHECK(fresh[0].data && *fresh[0].data == "fresh");
}

TEST(bounded_call_rethrows_and_notifies_after_the_result_is_in_place) {
    bool done_seen = false;
    std::mutex m;
    bounded::detail::MonoCond cv;
    bool notified = false;
    bounded::Call<int> c("", [] { return 42; }, [&] {
        std::lock_guard<std::mutex> g(m);
        notified = true;
        cv.notify_all();
    });
    {
        std::unique_lock<std::mutex> lk(m);
        cv.wait_until(lk, mono_ns() + 5000000000LL, [&] { return notified; });
        done_seen = c.done();  // done() is already true when notify runs
    }
    CHECK(notified && done_seen);
    CHECK(c.wait(mono_ns()) == std::optional<int>(42));
    bounded::Call<int> bad("", []() -> int { throw std::runtime_error("sysfs gone"); });
    std::string err;
    try {
        (void)bad.wait(mono_ns() + 1000000000LL);
    } catch (const std::runtime_error& e) {
        err = e.what();
    }
    CHECK_EQ(err, std::string("sysfs gone"));
    CHECK(!bounded::Call<int>().wait(mono_ns()));  // an empty call never blocks
}
