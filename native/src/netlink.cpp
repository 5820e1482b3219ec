#include "netop/netlink.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <linux/dcbnl.h>
#include <linux/if.h>
#include <linux/if_link.h>
#include <linux/netlink.h>
#include <linux/veth.h>
#include <net/if_arp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <set>

#include "netop/log.hpp"

#ifndef NETLINK_EXT_ACK
#define NETLINK_EXT_ACK 11
#endif
#ifndef NETLINK_CAP_ACK
#define NETLINK_CAP_ACK 10
#endif
#ifndef NLM_F_ACK_TLVS
#define NLM_F_ACK_TLVS 0x200
#endif
#ifndef NLM_F_CAPPED
#define NLM_F_CAPPED 0x100
#endif

namespace netop::nl {

// ---------------------------------------------------------------------------
// LinkInfo helpers
// ---------------------------------------------------------------------------
bool LinkInfo::up() const { return flags & IFF_UP; }
bool LinkInfo::lower_up() const { return flags & IFF_LOWER_UP; }

std::string LinkInfo::flags_str() const {
    std::vector<std::string> v;
    if (flags & IFF_UP) v.emplace_back("up");
    if (flags & IFF_BROADCAST) v.emplace_back("broadcast");
    if (flags & IFF_LOOPBACK) v.emplace_back("loopback");
    if (flags & IFF_POINTOPOINT) v.emplace_back("pointtopoint");
    if (flags & IFF_MULTICAST) v.emplace_back("multicast");
    if (flags & IFF_RUNNING) v.emplace_back("running");
    if (flags & IFF_PROMISC) v.emplace_back("promisc");
    if (flags & IFF_LOWER_UP) v.emplace_back("lower_up");
    return v.empty() ? "0" : join(v, "|");
}

std::string LinkInfo::operstate_str() const {
    static const char* names[] = {"unknown", "notpresent", "down", "lowerlayerdown", "testing", "dormant", "up"};
    return operstate < 7 ? names[operstate] : "unknown";
}

std::string RouteSpec::str() const {
    std::string s = dst.masked().str();
    if (gateway) s += " via " + gateway->str();
    s += strfmt(" dev#%d", ifindex);
    if (prefsrc) s += " src " + prefsrc->str();
    s += strfmt(" proto %u scope %u table %u", protocol, scope, table);
    return s;
}

std::string RuleSpec::str() const {
    return strfmt("from %s lookup %u priority %u", src.masked().str().c_str(), table, priority);
}

// ---------------------------------------------------------------------------
// Message builder
// ---------------------------------------------------------------------------
struct Rtnl::Msg {
    std::vector<uint8_t> buf;

    Msg(uint16_t type, uint16_t flags) {
        buf.resize(NLMSG_HDRLEN, 0);
        auto* h = hdr();
        h->nlmsg_type = type;
        h->nlmsg_flags = uint16_t(NLM_F_REQUEST | flags);
    }
    nlmsghdr* hdr() { return reinterpret_cast<nlmsghdr*>(buf.data()); }
    template <class T>
    size_t put(const T& t) {
        size_t off = buf.size();
        buf.resize(off + NLMSG_ALIGN(sizeof(T)), 0);
        std::memcpy(buf.data() + off, &t, sizeof(T));
        return off;
    }
    template <class T>
    T* at(size_t off) {
        return reinterpret_cast<T*>(buf.data() + off);
    }
    void attr(uint16_t type, const void* data, size_t len) {
        size_t off = buf.size();
        buf.resize(off + RTA_ALIGN(RTA_LENGTH(len)), 0);
        auto* a = reinterpret_cast<rtattr*>(buf.data() + off);
        a->rta_type = type;
        a->rta_len = uint16_t(RTA_LENGTH(len));
        if (len) std::memcpy(RTA_DATA(a), data, len);
    }
    void attr_u32(uint16_t type, uint32_t v) { attr(type, &v, 4); }
    void attr_ip(uint16_t type, Ipv4 ip) {
        uint8_t b[4];
        ip.to_net(b);
        attr(type, b, 4);
    }
    void attr_str(uint16_t type, const std::string& s) { attr(type, s.c_str(), s.size() + 1); }
    size_t nest_begin(uint16_t type) {
        size_t off = buf.size();
        attr(type, nullptr, 0);
        return off;
    }
    void nest_end(size_t off) {
        auto* a = reinterpret_cast<rtattr*>(buf.data() + off);
        a->rta_len = uint16_t(buf.size() - off);
    }
    void finalize(uint32_t seq) {
        hdr()->nlmsg_len = uint32_t(buf.size());
        hdr()->nlmsg_seq = seq;
    }
};

// ---------------------------------------------------------------------------
// Socket plumbing
// ---------------------------------------------------------------------------
static int open_rtnl_socket(uint32_t groups, uint32_t* portid) {
    int fd = ::socket(AF_NETLINK, SOCK_RAW | SOCK_CLOEXEC, NETLINK_ROUTE);
    if (fd < 0) throw_errno("socket(NETLINK_ROUTE)");
    int one = 1;
    ::setsockopt(fd, SOL_NETLINK, NETLINK_EXT_ACK, &one, sizeof one);
    ::setsockopt(fd, SOL_NETLINK, NETLINK_CAP_ACK, &one, sizeof one);
    int rcv = 1 << 20;
    ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof rcv);
    sockaddr_nl sa{};
    sa.nl_family = AF_NETLINK;
    sa.nl_groups = groups;
    if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
        int e = errno;
        ::close(fd);
        throw SysError(e, "bind(NETLINK_ROUTE)");
    }
    socklen_t sl = sizeof sa;
    ::getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &sl);
    if (portid) *portid = sa.nl_pid;
    return fd;
}

Rtnl::Rtnl() { fd_ = open_rtnl_socket(0, &portid_); }
Rtnl::~Rtnl() {
    if (fd_ >= 0) ::close(fd_);
}

std::string ext_ack_msg(const nlmsghdr* h) {
    // Extended ACK (NLM_F_ACK_TLVS): nlmsgerr, then the echoed request (unless NLM_F_CAPPED),
    // then attributes.  Every length comes from the peer, so each is checked against the bytes
    // the message actually has before it is used.
    if (h->nlmsg_len < NLMSG_LENGTH(sizeof(nlmsgerr)) || !(h->nlmsg_flags & NLM_F_ACK_TLVS)) return {};
    const auto* err = reinterpret_cast<const nlmsgerr*>(NLMSG_DATA(h));
    size_t off = NLMSG_HDRLEN + sizeof(nlmsgerr);
    if (!(h->nlmsg_flags & NLM_F_CAPPED)) {
        if (err->msg.nlmsg_len < sizeof(nlmsghdr)) return {};
        off += err->msg.nlmsg_len - sizeof(nlmsghdr);
    }
    off = NLMSG_ALIGN(off);  // the kernel pads the echoed request; a peer might not: copy, never cast
    const size_t end = h->nlmsg_len;
    const auto* base = reinterpret_cast<const uint8_t*>(h);
    while (off <= end && end - off >= sizeof(rtattr)) {
        rtattr a;
        std::memcpy(&a, base + off, sizeof a);
        if (a.rta_len < sizeof(rtattr) || a.rta_len > end - off) break;
        if (a.rta_type == 1 /* NLMSGERR_ATTR_MSG */) {
            const char* s = reinterpret_cast<const char*>(base + off + RTA_LENGTH(0));
            return std::string(s, strnlen(s, a.rta_len - RTA_LENGTH(0)));
        }
        off += RTA_ALIGN(a.rta_len);
    }
    return {};
}

static const char* msg_name(uint16_t t) {
    switch (t) {
        case RTM_NEWLINK: return "RTM_NEWLINK";
        case RTM_DELLINK: return "RTM_DELLINK";
        case RTM_GETLINK: return "RTM_GETLINK";
        case RTM_NEWADDR: return "RTM_NEWADDR";
        case RTM_DELADDR: return "RTM_DELADDR";
        case RTM_GETADDR: return "RTM_GETADDR";
        case RTM_NEWROUTE: return "RTM_NEWROUTE";
        case RTM_DELROUTE: return "RTM_DELROUTE";
        case RTM_GETROUTE: return "RTM_GETROUTE";
        case RTM_GETDCB: return "RTM_GETDCB";
        case RTM_SETDCB: return "RTM_SETDCB";
    }
    return "RTM_?";
}

void Rtnl::transact(Msg& m, const std::function<void(const nlmsghdr*)>& on_reply) {
    const uint32_t seq = seq_++;
    m.hdr()->nlmsg_flags |= NLM_F_ACK;
    m.finalize(seq);
    const uint16_t type = m.hdr()->nlmsg_type;
    ++rtts_;
    sockaddr_nl kernel{};
    kernel.nl_family = AF_NETLINK;
    for (;;) {
        ssize_t n = ::sendto(fd_, m.buf.data(), m.buf.size(), 0, reinterpret_cast<sockaddr*>(&kernel), sizeof kernel);
        if (n >= 0) break;
        if (errno == EINTR) continue;
        throw_errno(std::string("netlink send ") + msg_name(type));
    }
    alignas(nlmsghdr) static thread_local uint8_t buf[65536];
    for (;;) {
        ssize_t n = ::recv(fd_, buf, sizeof buf, 0);
        if (n < 0) {
            if (errno == EINTR) continue;
            throw_errno(std::string("netlink recv ") + msg_name(type));
        }
        long len = long(n);  // signed: NLMSG_NEXT must not wrap on a short final message
        for (auto* h = reinterpret_cast<nlmsghdr*>(buf); NLMSG_OK(h, len); h = NLMSG_NEXT(h, len)) {
            if (h->nlmsg_seq != seq) continue;  // stale reply to an earlier request
            if (h->nlmsg_type == NLMSG_ERROR) {
                const auto* err = reinterpret_cast<const nlmsgerr*>(NLMSG_DATA(h));
                if (err->error == 0) return;  // ACK
                std::string extra = ext_ack_msg(h);
                throw SysError(-err->error, std::string(msg_name(type)) + (extra.empty() ? "" : " (" + extra + ")"));
            }
            if (h->nlmsg_type == NLMSG_DONE) return;
            if (on_reply) on_reply(h);
        }
    }
}

void Rtnl::dump(Msg& m, const std::function<void(const nlmsghdr*)>& on_item) {
    for (int attempt = 0; attempt < 4; ++attempt) {
        const uint32_t seq = seq_++;
        m.hdr()->nlmsg_flags |= NLM_F_DUMP;
        m.finalize(seq);
        ++rtts_;
        sockaddr_nl kernel{};
        kernel.nl_family = AF_NETLINK;
        if (::sendto(fd_, m.buf.data(), m.buf.size(), 0, reinterpret_cast<sockaddr*>(&kernel), sizeof kernel) < 0)
            throw_errno(std::string("netlink dump send ") + msg_name(m.hdr()->nlmsg_type));
        std::vector<std::vector<uint8_t>> items;
        bool interrupted = false;
        alignas(nlmsghdr) static thread_local uint8_t buf[65536];
        for (bool done = false; !done;) {
            ssize_t n = ::recv(fd_, buf, sizeof buf, 0);
            if (n < 0) {
                if (errno == EINTR) continue;
                throw_errno("netlink dump recv");
            }
            long len = long(n);  // signed: NLMSG_NEXT must not wrap on a short final message
            for (auto* h = reinterpret_cast<nlmsghdr*>(buf); NLMSG_OK(h, len); h = NLMSG_NEXT(h, len)) {
                if (h->nlmsg_seq != seq) continue;
                if (h->nlmsg_flags & NLM_F_DUMP_INTR) interrupted = true;
                if (h->nlmsg_type == NLMSG_DONE) {
                    done = true;
                    break;
                }
                if (h->nlmsg_type == NLMSG_ERROR) {
                    const auto* err = reinterpret_cast<const nlmsgerr*>(NLMSG_DATA(h));
                    if (err->error == 0) {
                        done = true;
                        break;
                    }
                    throw SysError(-err->error, "netlink dump");
                }
                const auto* p = reinterpret_cast<const uint8_t*>(h);
                items.emplace_back(p, p + h->nlmsg_len);
            }
        }
        if (interrupted) continue;  // the table changed under the dump: retry for a consistent view
        for (auto& it : items) on_item(reinterpret_cast<const nlmsghdr*>(it.data()));
        return;
    }
    throw SysError(EAGAIN, "netlink dump kept being interrupted");
}

// ---------------------------------------------------------------------------
// Parsing
// ---------------------------------------------------------------------------
// A message must hold its fixed header before any of it is read: the kernel never sends less,
// but the parser must not trust that (fuzzing found the unchecked read).
template <class T>
static const T* fixed_header(const nlmsghdr* h, const char* what) {
    if (h->nlmsg_len < NLMSG_LENGTH(sizeof(T))) throw SysError(EBADMSG, std::string("truncated ") + what + " message");
    return reinterpret_cast<const T*>(NLMSG_DATA(h));
}

template <class F>
static void for_each_attr(const rtattr* a, size_t total, F&& f) {
    // Signed remaining length: RTA_NEXT subtracts the *aligned* attribute length, which can
    // exceed what is left for the last attribute; with an unsigned length that wraps and
    // RTA_OK would walk off the buffer (found by the netlink fuzz target).
    long len = total > size_t(1) << 30 ? 0 : long(total);
    for (; RTA_OK(a, len); a = RTA_NEXT(a, len)) f(a);
}

LinkInfo parse_link(const nlmsghdr* h) {
    LinkInfo li;
    const auto* ifi = fixed_header<ifinfomsg>(h, "link");
    li.index = ifi->ifi_index;
    li.flags = ifi->ifi_flags;
    size_t len = h->nlmsg_len - NLMSG_LENGTH(sizeof(ifinfomsg));
    for_each_attr(IFLA_RTA(ifi), len, [&](const rtattr* a) {
        switch (a->rta_type) {
            case IFLA_IFNAME:
                li.name.assign(reinterpret_cast<const char*>(RTA_DATA(a)), strnlen(reinterpret_cast<const char*>(RTA_DATA(a)), RTA_PAYLOAD(a)));
                break;
            case IFLA_MTU:
                if (RTA_PAYLOAD(a) >= 4) std::memcpy(&li.mtu, RTA_DATA(a), 4);
                break;
            case IFLA_ADDRESS:
                if (RTA_PAYLOAD(a) == 6) li.mac = MacAddr::from_bytes(reinterpret_cast<const uint8_t*>(RTA_DATA(a)));
                break;
            case IFLA_OPERSTATE:
                if (RTA_PAYLOAD(a) >= 1) li.operstate = *reinterpret_cast<const uint8_t*>(RTA_DATA(a));
                break;
            case IFLA_MASTER:
                if (RTA_PAYLOAD(a) >= 4) std::memcpy(&li.master, RTA_DATA(a), 4);
                break;
            case IFLA_LINKINFO:
                for_each_attr(reinterpret_cast<const rtattr*>(RTA_DATA(a)), RTA_PAYLOAD(a), [&](const rtattr* b) {
                    if (b->rta_type == IFLA_INFO_KIND)
                        li.kind.assign(reinterpret_cast<const char*>(RTA_DATA(b)), strnlen(reinterpret_cast<const char*>(RTA_DATA(b)), RTA_PAYLOAD(b)));
                });
                break;
        }
    });
    return li;
}

AddrInfo parse_addr(const nlmsghdr* h) {
    AddrInfo ai;
    const auto* ifa = fixed_header<ifaddrmsg>(h, "address");
    ai.ifindex = int(ifa->ifa_index);
    ai.family = ifa->ifa_family;
    ai.prefixlen = ifa->ifa_prefixlen;
    ai.scope = ifa->ifa_scope;
    bool have_local = false;
    size_t len = h->nlmsg_len - NLMSG_LENGTH(sizeof(ifaddrmsg));
    for_each_attr(IFA_RTA(ifa), len, [&](const rtattr* a) {
        if (ifa->ifa_family == AF_INET6 && a->rta_type == IFA_ADDRESS && RTA_PAYLOAD(a) == 16) {
            char buf[INET6_ADDRSTRLEN] = {};
            if (::inet_ntop(AF_INET6, RTA_DATA(a), buf, sizeof(buf))) ai.address6 = buf;
            return;
        }
        if (ifa->ifa_family != AF_INET) return;
        switch (a->rta_type) {
            case IFA_ADDRESS:
                if (RTA_PAYLOAD(a) == 4) ai.address = Ipv4::from_net(RTA_DATA(a));
                break;
            case IFA_LOCAL:
                if (RTA_PAYLOAD(a) == 4) {
                    ai.local = Ipv4::from_net(RTA_DATA(a));
                    have_local = true;
                }
                break;
            case IFA_LABEL:
                ai.label.assign(reinterpret_cast<const char*>(RTA_DATA(a)), strnlen(reinterpret_cast<const char*>(RTA_DATA(a)), RTA_PAYLOAD(a)));
                break;
        }
    });
    if (!have_local) ai.local = ai.address;
    return ai;
}

RouteInfo parse_route(const nlmsghdr* h) {
    RouteInfo r;
    const auto* rtm = fixed_header<rtmsg>(h, "route");
    r.dst.len = rtm->rtm_dst_len;
    r.scope = rtm->rtm_scope;
    r.protocol = rtm->rtm_protocol;
    r.table = rtm->rtm_table;
    r.type = rtm->rtm_type;
    size_t len = h->nlmsg_len - NLMSG_LENGTH(sizeof(rtmsg));
    for_each_attr(RTM_RTA(rtm), len, [&](const rtattr* a) {
        switch (a->rta_type) {
            case RTA_DST:
                if (RTA_PAYLOAD(a) == 4) r.dst.addr = Ipv4::from_net(RTA_DATA(a));
                break;
            case RTA_GATEWAY:
                if (RTA_PAYLOAD(a) == 4) r.gateway = Ipv4::from_net(RTA_DATA(a));
                break;
            case RTA_PREFSRC:
                if (RTA_PAYLOAD(a) == 4) r.prefsrc = Ipv4::from_net(RTA_DATA(a));
                break;
            case RTA_OIF:
                if (RTA_PAYLOAD(a) >= 4) std::memcpy(&r.ifindex, RTA_DATA(a), 4);
                break;
            case RTA_PRIORITY:
                if (RTA_PAYLOAD(a) >= 4) std::memcpy(&r.priority, RTA_DATA(a), 4);
                break;
            case RTA_MULTIPATH: {  // struct rtnexthop, each RTNH_ALIGNed; lengths bounds-checked
                const auto* p = static_cast<const uint8_t*>(RTA_DATA(a));
                size_t left = RTA_PAYLOAD(a);
                while (left >= sizeof(rtnexthop)) {
                    rtnexthop nh;
                    std::memcpy(&nh, p, sizeof nh);
                    if (nh.rtnh_len < sizeof(rtnexthop) || nh.rtnh_len > left) break;
                    if (nh.rtnh_ifindex > 0) r.nexthops.push_back(nh.rtnh_ifindex);
                    const size_t step = std::min<size_t>(RTNH_ALIGN(nh.rtnh_len), left);
                    p += step;
                    left -= step;
                }
                break;
            }
            case RTA_TABLE:
                if (RTA_PAYLOAD(a) >= 4) {
                    uint32_t t;
                    std::memcpy(&t, RTA_DATA(a), 4);
                    r.table = t;
                }
                break;
        }
    });
    return r;
}

// ---------------------------------------------------------------------------
// Operations
// ---------------------------------------------------------------------------
LinkInfo Rtnl::link_by_name(const std::string& name) {
    if (name.empty() || name.size() >= IFNAMSIZ) throw SysError(ENODEV, "link '" + name + "'");
    Msg m(RTM_GETLINK, 0);
    ifinfomsg ifi{};
    ifi.ifi_family = AF_UNSPEC;
    m.put(ifi);
    m.attr_str(IFLA_IFNAME, name);
    m.attr_u32(IFLA_EXT_MASK, RTEXT_FILTER_SKIP_STATS);
    std::optional<LinkInfo> out;
    try {
        transact(m, [&](const nlmsghdr* h) {
            if (h->nlmsg_type == RTM_NEWLINK) out = parse_link(h);
        });
    } catch (const SysError& e) {
        throw SysError(e.code(), "link '" + name + "' not found");
    }
    if (!out) throw SysError(ENODEV, "link '" + name + "' not found");
    return *out;
}

LinkInfo Rtnl::link_by_index(int ifindex) {
    Msg m(RTM_GETLINK, 0);
    ifinfomsg ifi{};
    ifi.ifi_family = AF_UNSPEC;
    ifi.ifi_index = ifindex;
    m.put(ifi);
    m.attr_u32(IFLA_EXT_MASK, RTEXT_FILTER_SKIP_STATS);
    std::optional<LinkInfo> out;
    transact(m, [&](const nlmsghdr* h) {
        if (h->nlmsg_type == RTM_NEWLINK) out = parse_link(h);
    });
    if (!out) throw SysError(ENODEV, strfmt("link #%d not found", ifindex));
    return *out;
}

std::optional<LinkStats> parse_link_stats(const nlmsghdr* h) {
    const auto* ifi = fixed_header<ifinfomsg>(h, "link");
    size_t len = h->nlmsg_len - NLMSG_LENGTH(sizeof(ifinfomsg));
    std::optional<LinkStats> s64, s32;
    for_each_attr(IFLA_RTA(ifi), len, [&](const rtattr* a) {
        if (a->rta_type == IFLA_STATS64 && RTA_PAYLOAD(a) >= sizeof(rtnl_link_stats64)) {
            rtnl_link_stats64 st;
            std::memcpy(&st, RTA_DATA(a), sizeof st);
            s64 = LinkStats{st.rx_packets, st.rx_bytes, st.multicast, st.rx_dropped};
        } else if (a->rta_type == IFLA_STATS && RTA_PAYLOAD(a) >= sizeof(rtnl_link_stats)) {
            rtnl_link_stats st;
            std::memcpy(&st, RTA_DATA(a), sizeof st);
            s32 = LinkStats{st.rx_packets, st.rx_bytes, st.multicast, st.rx_dropped};
        }
    });
    return s64 ? s64 : s32;
}

std::optional<LinkStats> Rtnl::link_stats(int ifindex) {
    Msg m(RTM_GETLINK, 0);
    ifinfomsg ifi{};
    ifi.ifi_family = AF_UNSPEC;
    ifi.ifi_index = ifindex;
    m.put(ifi);
    std::optional<LinkStats> out;
    try {
        transact(m, [&](const nlmsghdr* h) {
            if (h->nlmsg_type == RTM_NEWLINK) out = parse_link_stats(h);
        });
    } catch (const std::exception&) {  // counters are diagnostics: never fatal
        return std::nullopt;
    }
    return out;
}

std::optional<uint8_t> parse_dcb_u8(const nlmsghdr* h, uint16_t type) {
    const auto* d = fixed_header<dcbmsg>(h, "dcb");
    size_t len = h->nlmsg_len - NLMSG_LENGTH(sizeof(dcbmsg));
    std::optional<uint8_t> out;
    for_each_attr(reinterpret_cast<const rtattr*>(reinterpret_cast<const uint8_t*>(d) + NLMSG_ALIGN(sizeof(dcbmsg))),
                  len, [&](const rtattr* a) {
                      if (a->rta_type == type && RTA_PAYLOAD(a) >= 1) out = *static_cast<const uint8_t*>(RTA_DATA(a));
                  });
    return out;
}

// dcbnl answers a GET/SET with a message of the request's type carrying the result attribute,
// then the ACK; a driver without dcbnl_ops (or without the getter) fails the request with
// EOPNOTSUPP.
std::optional<uint8_t> Rtnl::dcbx_mode(const std::string& ifname) {
    Msg m(RTM_GETDCB, 0);
    dcbmsg d{};
    d.dcb_family = AF_UNSPEC;
    d.cmd = DCB_CMD_GDCBX;
    m.put(d);
    m.attr_str(DCB_ATTR_IFNAME, ifname);
    std::optional<uint8_t> out;
    try {
        transact(m, [&](const nlmsghdr* h) {
            if (h->nlmsg_type == RTM_GETDCB) out = parse_dcb_u8(h, DCB_ATTR_DCBX);
        });
    } catch (const SysError& e) {
        if (e.code() == EOPNOTSUPP || e.code() == ENODEV) return std::nullopt;
        throw;
    }
    return out;
}

bool Rtnl::set_dcbx_mode(const std::string& ifname, uint8_t mode) {
    Msg m(RTM_SETDCB, 0);
    dcbmsg d{};
    d.dcb_family = AF_UNSPEC;
    d.cmd = DCB_CMD_SDCBX;
    m.put(d);
    m.attr_str(DCB_ATTR_IFNAME, ifname);
    m.attr(DCB_ATTR_DCBX, &mode, 1);
    std::optional<uint8_t> status;
    transact(m, [&](const nlmsghdr* h) {
        if (h->nlmsg_type == RTM_SETDCB) status = parse_dcb_u8(h, DCB_ATTR_DCBX);
    });
    return status && *status == 0;
}

std::vector<LinkInfo> Rtnl::link_list() {
    Msg m(RTM_GETLINK, 0);
    ifinfomsg ifi{};
    ifi.ifi_family = AF_UNSPEC;
    m.put(ifi);
    m.attr_u32(IFLA_EXT_MASK, RTEXT_FILTER_SKIP_STATS);
    std::vector<LinkInfo> out;
    dump(m, [&](const nlmsghdr* h) {
        if (h->nlmsg_type == RTM_NEWLINK) out.push_back(parse_link(h));
    });
    return out;
}

std::vector<AddrInfo> Rtnl::addr_list(int ifindex, int family) {
    Msg m(RTM_GETADDR, 0);
    ifaddrmsg ifa{};
    ifa.ifa_family = uint8_t(family);
    m.put(ifa);
    std::vector<AddrInfo> out;
    dump(m, [&](const nlmsghdr* h) {
        if (h->nlmsg_type != RTM_NEWADDR) return;
        auto a = parse_addr(h);
        if (family != AF_UNSPEC && a.family != family) return;
        if (ifindex > 0 && a.ifindex != ifindex) return;
        out.push_back(a);
    });
    return out;
}

void Rtnl::addr_add(int ifindex, const Ipv4Prefix& addr) {
    Msg m(RTM_NEWADDR, NLM_F_CREATE | NLM_F_EXCL);
    ifaddrmsg ifa{};
    ifa.ifa_family = AF_INET;
    ifa.ifa_prefixlen = uint8_t(addr.len);
    ifa.ifa_scope = RT_SCOPE_UNIVERSE;
    ifa.ifa_index = uint32_t(ifindex);
    m.put(ifa);
    m.attr_ip(IFA_LOCAL, addr.addr);
    m.attr_ip(IFA_ADDRESS, addr.addr);
    if (addr.len < 31) m.attr_ip(IFA_BROADCAST, Ipv4{addr.addr.v | ~prefix_mask(addr.len)});
    transact(m, nullptr);
}

void Rtnl::addr_del(const AddrInfo& a) {
    Msg m(RTM_DELADDR, 0);
    ifaddrmsg ifa{};
    ifa.ifa_family = AF_INET;
    ifa.ifa_prefixlen = uint8_t(a.prefixlen);
    ifa.ifa_scope = a.scope;
    ifa.ifa_index = uint32_t(a.ifindex);
    m.put(ifa);
    m.attr_ip(IFA_LOCAL, a.local);
    m.attr_ip(IFA_ADDRESS, a.address);
    transact(m, nullptr);
}

void Rtnl::route_append(const RouteSpec& r) {
    Msg m(RTM_NEWROUTE, NLM_F_CREATE | NLM_F_APPEND);
    rtmsg rtm{};
    rtm.rtm_family = AF_INET;
    rtm.rtm_dst_len = uint8_t(r.dst.len);
    rtm.rtm_table = r.table < 256 ? uint8_t(r.table) : uint8_t(RT_TABLE_UNSPEC);
    rtm.rtm_protocol = r.protocol;
    rtm.rtm_scope = r.scope;
    rtm.rtm_type = r.type;
    m.put(rtm);
    m.attr_ip(RTA_DST, r.dst.network());
    if (r.gateway) m.attr_ip(RTA_GATEWAY, *r.gateway);
    if (r.prefsrc) m.attr_ip(RTA_PREFSRC, *r.prefsrc);
    if (r.ifindex > 0) m.attr_u32(RTA_OIF, uint32_t(r.ifindex));
    if (r.priority) m.attr_u32(RTA_PRIORITY, r.priority);
    m.attr_u32(RTA_TABLE, r.table);
    transact(m, nullptr);
}

void Rtnl::route_del(const RouteSpec& r) {
    Msg m(RTM_DELROUTE, 0);
    rtmsg rtm{};
    rtm.rtm_family = AF_INET;
    rtm.rtm_dst_len = uint8_t(r.dst.len);
    rtm.rtm_table = r.table < 256 ? uint8_t(r.table) : uint8_t(RT_TABLE_UNSPEC);
    rtm.rtm_scope = RT_SCOPE_NOWHERE;
    m.put(rtm);
    m.attr_ip(RTA_DST, r.dst.network());
    if (r.gateway) m.attr_ip(RTA_GATEWAY, *r.gateway);
    if (r.ifindex > 0) m.attr_u32(RTA_OIF, uint32_t(r.ifindex));
    m.attr_u32(RTA_TABLE, r.table);
    transact(m, nullptr);
}

std::vector<RouteInfo> Rtnl::route_list(uint32_t table) {
    Msg m(RTM_GETROUTE, 0);
    rtmsg rtm{};
    rtm.rtm_family = AF_INET;
    m.put(rtm);
    std::vector<RouteInfo> out;
    dump(m, [&](const nlmsghdr* h) {
        if (h->nlmsg_type != RTM_NEWROUTE) return;
        auto r = parse_route(h);
        if (table && r.table != table) return;
        out.push_back(r);
    });
    return out;
}

static void add_default_links(const RouteInfo& r, std::vector<int>& out) {
    if (r.dst.len != 0 || r.type != RTN_UNICAST || r.table == RT_TABLE_LOCAL) return;
    if (r.ifindex > 0) out.push_back(r.ifindex);
    out.insert(out.end(), r.nexthops.begin(), r.nexthops.end());
}

// Tables any packet may be looked up in: those of rules that look a table up and select nothing.
// nullopt: no rules to judge by (then every table counts, as before policy routing was read).
static std::optional<std::set<uint32_t>> lookup_all_tables(const std::vector<RuleSpec>& rules) {
    std::set<uint32_t> out;
    for (const auto& r : rules)
        if (r.action == 1 && !r.selective) out.insert(r.table);
    if (out.empty()) return std::nullopt;
    return out;
}

static std::optional<std::set<uint32_t>> global_tables(NetOps& ops) {
    try {
        return lookup_all_tables(ops.rule_list());
    } catch (const std::exception&) {
        return std::nullopt;  // conservative: every table's default route is an uplink
    }
}

std::vector<int> NetOps::default_route_links() {
    const auto global = global_tables(*this);
    std::vector<int> out;
    for (const auto& r : route_list(0))
        if (!global || global->count(r.table)) add_default_links(r, out);
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

std::vector<std::pair<int, uint32_t>> NetOps::policy_default_routes() {
    const auto global = global_tables(*this);
    std::vector<std::pair<int, uint32_t>> out;
    if (!global) return out;
    for (const auto& r : route_list(0)) {
        if (global->count(r.table)) continue;
        std::vector<int> links;
        add_default_links(r, links);
        for (int l : links) out.emplace_back(l, r.table);
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

std::vector<int> Rtnl::default_route_links() {
    std::vector<int> out = NetOps::default_route_links();
    // ::/0 too: a management NIC may carry only an IPv6 default route (SLAAC / RA).
    std::optional<std::set<uint32_t>> global6;
    try {
        global6 = lookup_all_tables(rule_list6());
    } catch (const std::exception&) {
    }
    Msg m(RTM_GETROUTE, 0);
    rtmsg rtm{};
    rtm.rtm_family = AF_INET6;
    m.put(rtm);
    try {
        dump(m, [&](const nlmsghdr* h) {
            if (h->nlmsg_type != RTM_NEWROUTE) return;
            auto r = parse_route(h);
            if (!global6 || global6->count(r.table)) add_default_links(r, out);
        });
    } catch (const SysError& e) {  // IPv6 disabled on the node (ipv6.disable=1)
        if (e.code() != EAFNOSUPPORT && e.code() != EOPNOTSUPP) throw;
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

namespace {
// FIB rule messages: struct fib_rule_hdr (linux/fib_rules.h) shares rtmsg's layout for the
// fields used here (family, dst_len, src_len, tos, table, res1, res2, action, flags).
constexpr uint16_t kFraSrc = 2, kFraPriority = 6, kFraTable = 15;  // FRA_SRC, FRA_PRIORITY, FRA_TABLE
constexpr uint16_t kFraProtocol = 21;                               // FRA_PROTOCOL (u8)
constexpr uint8_t kFrActToTbl = 1;                                  // FR_ACT_TO_TBL
// Attributes that make a rule match only some packets: FRA_DST 1, FRA_IIFNAME 3, FRA_FWMARK 10
// (when non-zero), FRA_OIFNAME 17, FRA_L3MDEV 19, FRA_UID_RANGE 20, FRA_IP_PROTO 22,
// FRA_SPORT_RANGE 23, FRA_DPORT_RANGE 24 (linux/fib_rules.h; FRA_SRC handled by src_len).
constexpr uint16_t kFraDst = 1, kFraIifname = 3, kFraFwmark = 10, kFraOifname = 17, kFraL3mdev = 19,
                   kFraUidRange = 20, kFraIpProto = 22, kFraSportRange = 23, kFraDportRange = 24;
constexpr uint32_t kFibRuleInvert = 0x2;  // FIB_RULE_INVERT
struct FibRuleHdr {
    uint8_t family, dst_len, src_len, tos, table, res1, res2, action;
    uint32_t flags;
};
}  // namespace

void Rtnl::rule_request(uint16_t type, uint16_t flags, const RuleSpec& r) {
    Msg m(type, flags);
    FibRuleHdr frh{};
    frh.family = AF_INET;
    frh.src_len = uint8_t(r.src.len);
    frh.table = r.table < 256 ? uint8_t(r.table) : uint8_t(RT_TABLE_UNSPEC);
    frh.action = kFrActToTbl;
    m.put(frh);
    if (r.src.len) m.attr_ip(kFraSrc, r.src.network());
    m.attr_u32(kFraTable, r.table);
    if (r.priority) m.attr_u32(kFraPriority, r.priority);
    if (r.protocol) m.attr(kFraProtocol, &r.protocol, 1);
    transact(m, nullptr);
}

void Rtnl::rule_add(const RuleSpec& r) { rule_request(RTM_NEWRULE, NLM_F_CREATE | NLM_F_EXCL, r); }

void Rtnl::rule_del(const RuleSpec& r) { rule_request(RTM_DELRULE, 0, r); }

std::optional<RuleSpec> parse_rule(const nlmsghdr* h) {
    if (h->nlmsg_len < NLMSG_LENGTH(sizeof(FibRuleHdr))) return std::nullopt;
    const auto* f = reinterpret_cast<const FibRuleHdr*>(NLMSG_DATA(h));
    RuleSpec r;
    r.src.len = f->src_len;
    r.table = f->table;
    r.action = f->action;
    r.selective = f->src_len || f->dst_len || f->tos || (f->flags & kFibRuleInvert);
    const auto* first = reinterpret_cast<const rtattr*>(reinterpret_cast<const char*>(f) + NLMSG_ALIGN(sizeof(FibRuleHdr)));
    const size_t len = h->nlmsg_len - NLMSG_LENGTH(NLMSG_ALIGN(sizeof(FibRuleHdr)));
    for_each_attr(first, len, [&](const rtattr* a) {
        switch (a->rta_type) {
            case kFraSrc:
                if (f->family == AF_INET && RTA_PAYLOAD(a) == 4) r.src.addr = Ipv4::from_net(RTA_DATA(a));
                break;
            case kFraPriority:
                if (RTA_PAYLOAD(a) >= 4) std::memcpy(&r.priority, RTA_DATA(a), 4);
                break;
            case kFraTable:
                if (RTA_PAYLOAD(a) >= 4) std::memcpy(&r.table, RTA_DATA(a), 4);
                break;
            case kFraProtocol:
                if (RTA_PAYLOAD(a) >= 1) r.protocol = *static_cast<const uint8_t*>(RTA_DATA(a));
                break;
            case kFraFwmark: {
                uint32_t mark = 0;
                if (RTA_PAYLOAD(a) >= 4) std::memcpy(&mark, RTA_DATA(a), 4);
                if (mark) r.selective = true;
                break;
            }
            case kFraDst:
            case kFraIifname:
            case kFraOifname:
            case kFraL3mdev:
            case kFraUidRange:
            case kFraIpProto:
            case kFraSportRange:
            case kFraDportRange:
                r.selective = true;
                break;
        }
    });
    return r;
}

std::vector<RuleSpec> Rtnl::dump_rules(uint8_t family) {
    Msg m(RTM_GETRULE, 0);
    FibRuleHdr frh{};
    frh.family = family;
    m.put(frh);
    std::vector<RuleSpec> out;
    dump(m, [&](const nlmsghdr* h) {
        if (h->nlmsg_type != RTM_NEWRULE) return;
        if (auto r = parse_rule(h)) out.push_back(*r);
    });
    return out;
}

std::vector<RuleSpec> Rtnl::rule_list() { return dump_rules(AF_INET); }

std::vector<RuleSpec> Rtnl::rule_list6() { return dump_rules(AF_INET6); }

void Rtnl::set_link(int ifindex, unsigned flags, unsigned change, const std::function<void(Msg&)>& attrs) {
    Msg m(RTM_NEWLINK, 0);
    ifinfomsg ifi{};
    ifi.ifi_family = AF_UNSPEC;
    ifi.ifi_index = ifindex;
    ifi.ifi_flags = flags;
    ifi.ifi_change = change;
    m.put(ifi);
    if (attrs) attrs(m);
    transact(m, nullptr);
}

void Rtnl::link_set_up(int ifindex) { set_link(ifindex, IFF_UP, IFF_UP, nullptr); }
void Rtnl::link_set_down(int ifindex) { set_link(ifindex, 0, IFF_UP, nullptr); }
void Rtnl::link_set_mtu(int ifindex, int mtu) {
    set_link(ifindex, 0, 0, [&](Msg& m) { m.attr_u32(IFLA_MTU, uint32_t(mtu)); });
}
void Rtnl::link_set_mac(int ifindex, const MacAddr& mac) {
    set_link(ifindex, 0, 0, [&](Msg& m) { m.attr(IFLA_ADDRESS, mac.b.data(), 6); });
}
void Rtnl::link_set_name(int ifindex, const std::string& name) {
    set_link(ifindex, 0, 0, [&](Msg& m) { m.attr_str(IFLA_IFNAME, name); });
}
void Rtnl::link_set_netns_fd(int ifindex, int netns_fd) {
    set_link(ifindex, 0, 0, [&](Msg& m) { m.attr_u32(IFLA_NET_NS_FD, uint32_t(netns_fd)); });
}
void Rtnl::link_set_netns_pid(int ifindex, int pid) {
    set_link(ifindex, 0, 0, [&](Msg& m) { m.attr_u32(IFLA_NET_NS_PID, uint32_t(pid)); });
}

void Rtnl::veth_add(const std::string& name, const std::string& peer) {
    Msg m(RTM_NEWLINK, NLM_F_CREATE | NLM_F_EXCL);
    ifinfomsg ifi{};
    ifi.ifi_family = AF_UNSPEC;
    m.put(ifi);
    m.attr_str(IFLA_IFNAME, name);
    size_t li = m.nest_begin(IFLA_LINKINFO);
    m.attr_str(IFLA_INFO_KIND, "veth");
    size_t data = m.nest_begin(IFLA_INFO_DATA);
    size_t peer_nest = m.nest_begin(VETH_INFO_PEER);
    ifinfomsg pifi{};
    pifi.ifi_family = AF_UNSPEC;
    m.put(pifi);
    m.attr_str(IFLA_IFNAME, peer);
    m.nest_end(peer_nest);
    m.nest_end(data);
    m.nest_end(li);
    transact(m, nullptr);
}

void Rtnl::link_add(const std::string& name, const std::string& kind) {
    Msg m(RTM_NEWLINK, NLM_F_CREATE | NLM_F_EXCL);
    ifinfomsg ifi{};
    ifi.ifi_family = AF_UNSPEC;
    m.put(ifi);
    m.attr_str(IFLA_IFNAME, name);
    size_t li = m.nest_begin(IFLA_LINKINFO);
    m.attr_str(IFLA_INFO_KIND, kind);
    m.nest_end(li);
    transact(m, nullptr);
}

void Rtnl::link_set_master(int ifindex, int master) {
    set_link(ifindex, 0, 0, [&](Msg& m) { m.attr_u32(IFLA_MASTER, uint32_t(master)); });
}

std::optional<LinkInfo> Rtnl::link_by_ifindex(int ifindex) {
    try {
        return link_by_index(ifindex);
    } catch (const SysError& e) {
        if (e.code() == ENODEV) return std::nullopt;
        throw;
    }
}

void Rtnl::link_del(int ifindex) {
    Msg m(RTM_DELLINK, 0);
    ifinfomsg ifi{};
    ifi.ifi_family = AF_UNSPEC;
    ifi.ifi_index = ifindex;
    m.put(ifi);
    transact(m, nullptr);
}

// ---------------------------------------------------------------------------
// Link watcher (RTNLGRP_LINK multicast)
// ---------------------------------------------------------------------------
namespace {
class RtnlLinkWatcher final : public LinkWatcher {
   public:
    RtnlLinkWatcher() { fd_ = open_rtnl_socket(RTMGRP_LINK, nullptr); }
    ~RtnlLinkWatcher() override { ::close(fd_); }
    int fd() const override { return fd_; }

    std::vector<LinkEvent> wait(int64_t deadline) override {
        std::vector<LinkEvent> out;
        alignas(nlmsghdr) uint8_t buf[32768];
        for (;;) {
            int64_t now = mono_ns();
            int timeout_ms = deadline <= now ? 0 : int((deadline - now + 999999) / 1000000);
            pollfd p{fd_, POLLIN, 0};
            int r = ::poll(&p, 1, out.empty() ? timeout_ms : 0);
            if (r < 0) {
                if (errno == EINTR) continue;
                throw_errno("poll(link watcher)");
            }
            if (r == 0) return out;
            ssize_t n = ::recv(fd_, buf, sizeof buf, MSG_DONTWAIT);
            if (n < 0) {
                if (errno == EINTR || errno == EAGAIN) continue;
                if (errno == ENOBUFS) continue;  // overrun: events lost; caller re-reads state
                throw_errno("recv(link watcher)");
            }
            long len = long(n);  // signed: NLMSG_NEXT must not wrap on a short final message
            for (auto* h = reinterpret_cast<nlmsghdr*>(buf); NLMSG_OK(h, len); h = NLMSG_NEXT(h, len)) {
                if (h->nlmsg_type != RTM_NEWLINK && h->nlmsg_type != RTM_DELLINK) continue;
                LinkEvent ev;
                ev.deleted = h->nlmsg_type == RTM_DELLINK;
                ev.link = parse_link(h);
                out.push_back(std::move(ev));
            }
        }
    }

   private:
    int fd_ = -1;
};
}  // namespace

std::unique_ptr<LinkWatcher> Rtnl::subscribe_links() { return std::make_unique<RtnlLinkWatcher>(); }

}  // namespace netop::nl

