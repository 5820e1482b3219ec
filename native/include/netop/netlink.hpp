// Raw rtnetlink client (NETLINK_ROUTE) — no libnl, no external deps.
//
// Replaces the reference's vishvananda/netlink function table
// (reference cmd/discover/network.go:41-63).  `NetOps` is the injectable
// interface (the reference swaps `networkLink.*` function pointers in tests,
// network_test.go:276,364-366); `Rtnl` is the real implementation over one
// ACKed request socket, and `LinkWatcher` a separate RTNLGRP_LINK multicast
// socket used to wait for link-state echoes (network.go:242-283).
#pragma once

#include <linux/rtnetlink.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "netop/common.hpp"

namespace netop::nl {

struct LinkInfo {
    int index = 0;
    std::string name;
    unsigned flags = 0;  // IFF_*
    int mtu = 0;
    MacAddr mac;
    uint8_t operstate = 0;  // IF_OPER_*
    std::string kind;       // IFLA_INFO_KIND ("veth", ...) when present
    int master = 0;
    bool up() const;
    bool lower_up() const;
    std::string flags_str() const;  // "up|broadcast|multicast" (Go net.Flags.String() style)
    std::string operstate_str() const;
};

// Receive counters of a link (IFLA_STATS64): used to tell a NIC that hears nothing from one
// that hears traffic but no LLDP (a NIC-firmware LLDP agent consuming the frames).
struct LinkStats {
    uint64_t rx_packets = 0;
    uint64_t rx_bytes = 0;
    uint64_t multicast = 0;
    uint64_t rx_dropped = 0;
};

struct AddrInfo {
    int ifindex = 0;
    int family = 0;
    Ipv4 address;  // IFA_ADDRESS (peer for p2p links)
    Ipv4 local;    // IFA_LOCAL
    int prefixlen = 0;
    uint8_t scope = 0;
    std::string label;
    std::string address6;  // AF_INET6: the address in text form ("fd00::5"); empty for IPv4
    Ipv4Prefix prefix() const { return Ipv4Prefix{local, prefixlen}; }
};

struct RouteSpec {
    int ifindex = 0;
    Ipv4Prefix dst{};
    std::optional<Ipv4> gateway;
    std::optional<Ipv4> prefsrc;
    uint8_t scope = RT_SCOPE_UNIVERSE;
    uint8_t protocol = RTPROT_BOOT;  // vishvananda/netlink's NewRtMsg default
    uint32_t table = RT_TABLE_MAIN;  // RTA_TABLE: ids above 255 do not fit rtm_table
    uint8_t type = RTN_UNICAST;
    uint32_t priority = 0;
    // Listing only: the output interfaces of a multipath route's next hops (RTA_MULTIPATH).
    std::vector<int> nexthops;
    std::string str() const;
};

using RouteInfo = RouteSpec;

// Source-address policy rule (`ip rule add from <src> lookup <table> priority <priority>`),
// used for per-rail routing tables.
struct RuleSpec {
    Ipv4Prefix src{};
    uint32_t table = 0;
    uint32_t priority = 0;
    // FRA_PROTOCOL (Linux >= 4.17): who installed the rule.  0 = unspecified (matches any on
    // delete).  The agent tags its rail rules so it only ever removes rules it added.
    uint8_t protocol = 0;
    // Listing only.  action: FR_ACT_* (1 = look up `table`).  selective: the rule matches only
    // some packets (a source or destination prefix, TOS, in/out interface, fwmark, L3 master
    // device, uid, IP protocol or port range, or an inverted match); `from all lookup main`
    // is not.
    uint8_t action = 1;
    bool selective = false;
    bool operator==(const RuleSpec& o) const {
        return src.masked() == o.src.masked() && table == o.table && priority == o.priority && protocol == o.protocol;
    }
    std::string str() const;
};

struct LinkEvent {
    bool deleted = false;
    LinkInfo link;
};

class LinkWatcher {
   public:
    virtual ~LinkWatcher() = default;
    // Blocks until at least one event or the absolute CLOCK_MONOTONIC deadline; returns
    // all events read (possibly empty on timeout).
    virtual std::vector<LinkEvent> wait(int64_t deadline_mono_ns) = 0;
    // Pollable descriptor that becomes readable when events are pending (-1 if none).
    virtual int fd() const { return -1; }
};

// The injectable operation table.  Every method throws SysError on failure.
class NetOps {
   public:
    virtual ~NetOps() = default;
    virtual LinkInfo link_by_name(const std::string& name) = 0;
    virtual std::vector<AddrInfo> addr_list(int ifindex, int family) = 0;  // family: AF_INET / AF_UNSPEC
    virtual void addr_add(int ifindex, const Ipv4Prefix& addr) = 0;
    virtual void addr_del(const AddrInfo& addr) = 0;
    virtual void route_append(const RouteSpec& r) = 0;
    virtual void route_del(const RouteSpec& r) = 0;
    // Rules: add fails with EEXIST for an identical rule (NLM_F_EXCL); list returns IPv4 rules.
    virtual void rule_add(const RuleSpec& r) = 0;
    virtual void rule_del(const RuleSpec& r) = 0;
    virtual std::vector<RuleSpec> rule_list() = 0;
    // IPv4 routes of one table (0 = every table).
    virtual std::vector<RouteSpec> route_list(uint32_t table) = 0;
    virtual void link_set_up(int ifindex) = 0;
    virtual void link_set_down(int ifindex) = 0;
    virtual void link_set_mtu(int ifindex, int mtu) = 0;
    virtual std::unique_ptr<LinkWatcher> subscribe_links() = 0;
    // Receive counters; nullopt where the source has none (fakes, old kernels).
    virtual std::optional<LinkStats> link_stats(int ifindex) {
        (void)ifindex;
        return std::nullopt;
    }
    // Interfaces a default route (0.0.0.0/0, and ::/0 where the source lists IPv6) leaves
    // through, in a table that every packet the node sends may be looked up in (reached by a
    // rule that selects nothing: main and default, normally): the node's own uplinks, which the
    // agent never flushes or re-MTUs.  A default route in a table that only selective rules reach
    // (per-NIC source routing, "from 10.1.0.0/16 lookup 101") is not an uplink: see
    // policy_default_routes().  Without the rules (unreadable) every table but local counts.
    // The base implementation reads route_list(0) and rule_list().
    virtual std::vector<int> default_route_links();
    // (ifindex, table) of the IPv4 default routes that only selective rules reach.
    std::vector<std::pair<int, uint32_t>> policy_default_routes();
    // The link with this ifindex (a bond / bridge master, ...); nullopt when there is none or the
    // source cannot look links up by index.
    virtual std::optional<LinkInfo> link_by_ifindex(int ifindex) {
        (void)ifindex;
        return std::nullopt;
    }
};

class Rtnl final : public NetOps {
   public:
    Rtnl();
    ~Rtnl() override;
    Rtnl(const Rtnl&) = delete;
    Rtnl& operator=(const Rtnl&) = delete;

    LinkInfo link_by_name(const std::string& name) override;
    std::vector<AddrInfo> addr_list(int ifindex, int family) override;
    void addr_add(int ifindex, const Ipv4Prefix& addr) override;
    void addr_del(const AddrInfo& addr) override;
    void route_append(const RouteSpec& r) override;
    void route_del(const RouteSpec& r) override;
    void rule_add(const RuleSpec& r) override;
    void rule_del(const RuleSpec& r) override;
    std::vector<RuleSpec> rule_list() override;
    std::vector<RuleSpec> rule_list6();  // IPv6 rules (action, table, selective)
    void link_set_up(int ifindex) override;
    void link_set_down(int ifindex) override;
    void link_set_mtu(int ifindex, int mtu) override;
    std::unique_ptr<LinkWatcher> subscribe_links() override;
    std::optional<LinkStats> link_stats(int ifindex) override;
    std::vector<int> default_route_links() override;  // IPv4 and IPv6
    std::optional<LinkInfo> link_by_ifindex(int ifindex) override;

    // Extra operations (harness / diagnostics; not part of the injectable table).
    LinkInfo link_by_index(int ifindex);
    std::vector<LinkInfo> link_list();
    std::vector<RouteInfo> route_list(uint32_t table = RT_TABLE_MAIN) override;
    void veth_add(const std::string& name, const std::string& peer);
    // A link of a kind that needs no IFLA_INFO_DATA ("bridge", "dummy", ...).
    void link_add(const std::string& name, const std::string& kind);
    void link_set_master(int ifindex, int master);  // 0 = release from its master
    void link_del(int ifindex);
    void link_set_netns_fd(int ifindex, int netns_fd);
    void link_set_netns_pid(int ifindex, int pid);
    void link_set_mac(int ifindex, const MacAddr& mac);
    void link_set_name(int ifindex, const std::string& name);

    // DCB netlink (dcbnl, RTM_GETDCB / RTM_SETDCB): the DCBX mode of a NIC as DCB_CAP_DCBX_*
    // bits.  nullopt when the driver has no DCB interface (EOPNOTSUPP: veth, virtio, ...).
    // Reading needs no privileges; setting needs CAP_NET_ADMIN.
    std::optional<uint8_t> dcbx_mode(const std::string& ifname);
    // false when the driver refused the mode (dcbnl status byte != 0).  Throws SysError.
    bool set_dcbx_mode(const std::string& ifname, uint8_t mode);

    // Number of request round trips done on this socket (observability / bench).
    uint64_t round_trips() const { return rtts_; }

   private:
    struct Msg;
    void rule_request(uint16_t type, uint16_t flags, const RuleSpec& r);
    void transact(Msg& m, const std::function<void(const nlmsghdr*)>& on_reply);
    void dump(Msg& m, const std::function<void(const nlmsghdr*)>& on_item);
    std::vector<RuleSpec> dump_rules(uint8_t family);
    void set_link(int ifindex, unsigned flags, unsigned change, const std::function<void(Msg&)>& attrs);

    int fd_ = -1;
    uint32_t seq_ = 1;
    uint32_t portid_ = 0;
    uint64_t rtts_ = 0;
};

// Parses an RTM_NEWLINK/RTM_DELLINK payload.
LinkInfo parse_link(const nlmsghdr* h);
// Parses an RTM_NEWROUTE payload (IPv4 fields; dst_len, table, type, protocol, output interfaces
// of any family, RTA_MULTIPATH next hops included).  Bounds-checked like parse_link.
RouteInfo parse_route(const nlmsghdr* h);
// Parses an RTM_NEWADDR payload: IPv4 fields, or for AF_INET6 the address in text form
// (address6).  Bounds-checked like parse_link.
AddrInfo parse_addr(const nlmsghdr* h);
// Parses an RTM_NEWRULE payload (struct fib_rule_hdr + FRA_* attributes): table (FRA_TABLE
// over the header's), priority, protocol, action, the IPv4 source, and whether any selector is
// present (RuleSpec::selective).  nullopt when the message is too short.  Bounds-checked like
// parse_link.
std::optional<RuleSpec> parse_rule(const nlmsghdr* h);
// IFLA_STATS64 (else IFLA_STATS) of an RTM_NEWLINK message; nullopt when it carries neither.
std::optional<LinkStats> parse_link_stats(const nlmsghdr* h);
// The NLMSGERR_ATTR_MSG string of an extended ACK (NLMSG_ERROR with NLM_F_ACK_TLVS); "" if
// absent.  `h->nlmsg_len` bytes must be readable; every inner length is bounds-checked.
std::string ext_ack_msg(const nlmsghdr* h);
// The u8 attribute `type` of an RTM_GETDCB / RTM_SETDCB reply (dcbmsg header); nullopt if
// absent.  Bounds-checked like parse_link.
std::optional<uint8_t> parse_dcb_u8(const nlmsghdr* h, uint16_t type);

}  // namespace netop::nl
