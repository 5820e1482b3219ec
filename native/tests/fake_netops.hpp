// In-memory NetOps with per-operation fault injection — the C++ counterpart of the
// reference's function-table fakes (reference cmd/discover/network_test.go:276,364-366,
// 405,429,516-519,555-558,595,605).
#pragma once

#include <linux/if.h>
#include <sys/socket.h>

#include <algorithm>
#include <deque>
#include <functional>
#include <map>
#include <set>

#include "netop/netlink.hpp"

struct FakeNetOps : netop::nl::NetOps {
    std::map<std::string, netop::nl::LinkInfo> links;
    std::vector<netop::nl::AddrInfo> addrs;
    std::vector<netop::nl::RouteSpec> routes;
    std::vector<netop::nl::RuleSpec> rules;
    std::set<std::string> fail;  // op names that throw: "link_by_name", "addr_list", ...
    int fail_errno = EPERM;
    bool echo_links = true;      // emit RTM_NEWLINK on set up/down
    std::deque<netop::nl::LinkEvent> events;
    std::map<std::string, int> calls;

    // Cable state: a link that is admin-up has IFF_LOWER_UP unless its name is listed here.
    std::set<std::string> no_carrier;
    void add_link(const std::string& name, int index, const char* mac, bool up) {
        netop::nl::LinkInfo l;
        l.name = name;
        l.index = index;
        l.mac = *netop::MacAddr::parse(mac);
        l.flags = IFF_BROADCAST | IFF_MULTICAST | (up ? IFF_UP | IFF_LOWER_UP : 0);
        l.mtu = 1500;
        links[name] = l;
    }
    // The cable is plugged in (or pulled): carrier follows, with the kernel's RTM_NEWLINK.
    void set_carrier(const std::string& name, bool on) {
        auto& l = links[name];
        if (on) {
            no_carrier.erase(name);
            if (l.flags & IFF_UP) l.flags |= IFF_LOWER_UP;
        } else {
            no_carrier.insert(name);
            l.flags &= ~unsigned(IFF_LOWER_UP);
        }
        events.push_back({false, l});
    }
    netop::nl::LinkInfo* by_index(int idx) {
        for (auto& [n, l] : links)
            if (l.index == idx) return &l;
        return nullptr;
    }
    std::function<void(const std::string&)> on_op;     // runs at every operation, before it acts
    std::function<void(const std::string&)> after_op;  // after an address change took effect
    void maybe_fail(const std::string& op) {
        ++calls[op];
        if (on_op) on_op(op);
        if (fail.count(op)) throw netop::SysError(fail_errno, "injected " + op);
    }
    std::optional<netop::nl::LinkInfo> link_by_ifindex(int ifindex) override {
        maybe_fail("link_by_ifindex");
        if (auto* l = by_index(ifindex)) return *l;
        return std::nullopt;
    }
    netop::nl::LinkInfo link_by_name(const std::string& name) override {
        maybe_fail("link_by_name");
        auto it = links.find(name);
        if (it == links.end()) throw netop::SysError(ENODEV, "link '" + name + "' not found");
        return it->second;
    }
    std::vector<netop::nl::AddrInfo> addr_list(int ifindex, int family) override {
        maybe_fail("addr_list");
        std::vector<netop::nl::AddrInfo> out;
        for (auto& a : addrs) {
            // (entries without a family are IPv4, as the tests write them)
            const bool v6 = a.family == AF_INET6;
            if (a.ifindex == ifindex && (family == AF_UNSPEC || (family == AF_INET6) == v6)) out.push_back(a);
        }
        return out;
    }
    void addr_add(int ifindex, const netop::Ipv4Prefix& p) override {
        maybe_fail("addr_add");
        for (auto& a : addrs)
            if (a.ifindex == ifindex && a.local == p.addr) throw netop::SysError(EEXIST, "addr exists");
        netop::nl::AddrInfo a;
        a.ifindex = ifindex;
        a.family = AF_INET;
        a.local = a.address = p.addr;
        a.prefixlen = p.len;
        addrs.push_back(a);
        // the kernel's connected route
        netop::nl::RouteSpec r;
        r.ifindex = ifindex;
        r.dst = p.masked();
        r.prefsrc = p.addr;
        r.protocol = RTPROT_KERNEL;
        r.scope = RT_SCOPE_LINK;
        routes.push_back(r);
        if (after_op) after_op("addr_add");
    }
    void addr_del(const netop::nl::AddrInfo& a) override {
        maybe_fail("addr_del");
        auto it = std::find_if(addrs.begin(), addrs.end(), [&](const netop::nl::AddrInfo& x) {
            return x.ifindex == a.ifindex && x.local == a.local;
        });
        if (it == addrs.end()) throw netop::SysError(EADDRNOTAVAIL, "no such address");
        routes.erase(std::remove_if(routes.begin(), routes.end(), [&](const netop::nl::RouteSpec& r) {
                         return r.ifindex == a.ifindex && (r.prefsrc == std::optional<netop::Ipv4>(a.local) ||
                                                            (r.gateway && netop::Ipv4Prefix{a.local, a.prefixlen}.contains(*r.gateway)));
                     }),
                     routes.end());
        addrs.erase(it);
        if (after_op) after_op("addr_del");
    }
    void route_append(const netop::nl::RouteSpec& r) override {
        maybe_fail("route_append");
        for (auto& x : routes)
            if (x.ifindex == r.ifindex && x.dst.masked() == r.dst.masked() && x.gateway == r.gateway && x.table == r.table)
                throw netop::SysError(EEXIST, "route exists");
        routes.push_back(r);
    }
    void route_del(const netop::nl::RouteSpec& r) override {
        maybe_fail("route_del");
        auto it = std::find_if(routes.begin(), routes.end(), [&](const netop::nl::RouteSpec& x) {
            return x.dst.masked() == r.dst.masked() && x.table == r.table && (!r.gateway || x.gateway == r.gateway) &&
                   (r.ifindex <= 0 || x.ifindex == r.ifindex);
        });
        if (it == routes.end()) throw netop::SysError(ESRCH, "no such route");
        routes.erase(it);
    }
    void rule_add(const netop::nl::RuleSpec& r) override {
        maybe_fail("rule_add");
        if (std::find(rules.begin(), rules.end(), r) != rules.end()) throw netop::SysError(EEXIST, "rule exists");
        rules.push_back(r);
    }
    void rule_del(const netop::nl::RuleSpec& r) override {
        maybe_fail("rule_del");
        auto it = std::find(rules.begin(), rules.end(), r);
        if (it == rules.end()) throw netop::SysError(ENOENT, "no such rule");
        rules.erase(it);
    }
    std::vector<netop::nl::RuleSpec> rule_list() override {
        maybe_fail("rule_list");
        return rules;
    }
    std::vector<netop::nl::RouteSpec> route_list(uint32_t table) override {
        maybe_fail("route_list");
        std::vector<netop::nl::RouteSpec> out;
        for (auto& r : routes)
            if (!table || r.table == table) out.push_back(r);
        return out;
    }
    void set_flag(int ifindex, bool up) {
        auto* l = by_index(ifindex);
        if (!l) throw netop::SysError(ENODEV, "no link");
        l->flags = up ? (l->flags | IFF_UP) : (l->flags & ~unsigned(IFF_UP | IFF_LOWER_UP));
        if (up && !no_carrier.count(l->name)) l->flags |= IFF_LOWER_UP;
        if (echo_links) events.push_back({false, *l});
    }
    void link_set_up(int ifindex) override {
        maybe_fail("link_set_up");
        set_flag(ifindex, true);
    }
    void link_set_down(int ifindex) override {
        maybe_fail("link_set_down");
        set_flag(ifindex, false);
    }
    void link_set_mtu(int ifindex, int mtu) override {
        maybe_fail("link_set_mtu");
        if (auto* l = by_index(ifindex)) l->mtu = mtu;
    }
    struct Watcher : netop::nl::LinkWatcher {
        FakeNetOps* f;
        explicit Watcher(FakeNetOps* ff) : f(ff) {}
        std::vector<netop::nl::LinkEvent> wait(int64_t) override {
            std::vector<netop::nl::LinkEvent> out(f->events.begin(), f->events.end());
            f->events.clear();
            return out;
        }
    };
    // Receive counters: rx[ifindex] is returned and then advanced by rx_step[ifindex] per call
    // (traffic arriving while the agent waits); links without an entry have no counters.
    std::map<int, uint64_t> rx, rx_step;
    std::optional<netop::nl::LinkStats> link_stats(int ifindex) override {
        maybe_fail("link_stats");
        auto it = rx.find(ifindex);
        if (it == rx.end()) return std::nullopt;
        netop::nl::LinkStats s;
        s.rx_packets = it->second;
        it->second += rx_step[ifindex];
        return s;
    }
    std::unique_ptr<netop::nl::LinkWatcher> subscribe_links() override {
        maybe_fail("subscribe_links");
        return std::make_unique<Watcher>(this);
    }
};
