// libFuzzer targets for every parser that reads bytes the agent does not control.
//
//   lldp      frames from the switch (AF_PACKET) — untrusted, L2-adjacent attacker — and the
//             LLDP cache lines made from them
//   dbus      messages from the system bus peer
//   portdesc  the switch's Port Description string (operator-configured, still untrusted), the
//             agent's --fw-lldp-state record (a hostPath file), and amdgpu's gpu_metrics blob
//   netlink   RTM_NEWLINK / NEWROUTE / NEWRULE / NEWADDR / DCB / extended-ACK payloads (kernel,
//             but parsed with length arithmetic)
//   arp       ARP payloads from the switch port (--verify-peers) — untrusted, L2-adjacent
//
// Built by `make fuzz-native` with amdclang++ -fsanitize=fuzzer,address,undefined (one binary
// per target, selected by NETOP_FUZZ_TARGET at compile time).  Each target must never crash,
// hang or trip a sanitizer on any input.
#include <linux/dcbnl.h>
#include <linux/netlink.h>
#include <linux/rtnetlink.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "netop/arp.hpp"
#include "netop/artifacts.hpp"
#include "netop/dbus.hpp"
#include "netop/ethtool.hpp"
#include "netop/l3.hpp"
#include "netop/lldp.hpp"
#include "netop/netlink.hpp"
#include "netop/topology.hpp"

using namespace netop;

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
#if NETOP_FUZZ_TARGET == 1
    lldp::DecodeError err;
    auto f = lldp::decode(data, size, &err);
    if (f) {
        // Whatever decodes must re-encode and decode to the same fields.
        auto bytes = lldp::encode(*f);
        auto again = lldp::decode(bytes.data(), bytes.size());
        if (!again || again->port_description != f->port_description || again->ttl != f->ttl) __builtin_trap();
        if (again->max_frame_size() != f->max_frame_size()) __builtin_trap();  // 802.3 org TLV survives
        // The LLDP cache stores the switch's strings: whatever they hold, they stay inside their
        // own fields of their own NIC's line (no forged entry for another NIC).
        artifacts::LldpCacheEntry mine{"02:00:00:00:00:01", "ens0", 1, "", f->system_name.value_or(""),
                                       f->port_id_str(), f->port_description.value_or("")};
        artifacts::LldpCacheEntry other{"02:00:00:00:00:02", "ens1", 2, "", "leaf", "swp1", "x 10.0.0.2/30"};
        auto back = artifacts::decode_lldp_cache(artifacts::encode_lldp_cache({mine, other}));
        if (back.size() != 2 || back[0].ifname != "ens0" || back[1].ifname != "ens1" ||
            back[1].port_description != other.port_description || back[0].unix_s != 1)
            __builtin_trap();
    }
#elif NETOP_FUZZ_TARGET == 2
    dbus::Message m;
    size_t used = 0;
    try {
        used = dbus::unmarshal(data, size, &m);
    } catch (const std::exception&) {
        return 0;
    }
    if (used > size) __builtin_trap();
#elif NETOP_FUZZ_TARGET == 3
    std::string s(reinterpret_cast<const char*>(data), size);
    for (auto p : {l3::TokenPolicy::Compat, l3::TokenPolicy::CompatThenLast, l3::TokenPolicy::AnyToken}) {
        std::string err;
        auto a = l3::parse_port_description(s, p, &err);
        if (a && (a->local.v ^ a->peer.v) != 3u) __builtin_trap();
    }
    // The firmware-LLDP record on the node (--fw-lldp-state, a hostPath file): whatever decodes
    // re-encodes to a record that decodes to the same originals.
    auto recs = ethtool::decode_state(s);
    auto again = ethtool::decode_state(ethtool::encode_state(recs));
    if (again.size() != recs.size()) __builtin_trap();
    for (size_t i = 0; i < recs.size(); ++i)
        if (again[i].ifname != recs[i].ifname || again[i].changed != recs[i].changed ||
            again[i].original_bits != recs[i].original_bits || again[i].dcbx_changed != recs[i].dcbx_changed ||
            again[i].dcbx != recs[i].dcbx)
            __builtin_trap();
    // The GPU's gpu_metrics blob (sysfs): decoded only at a known revision, never read past its end.
    auto h = topo::parse_gpu_metrics(s);
    if (h.known && (h.status.size() != size_t(topo::kMaxXgmiLinks) || h.links_up() + h.links_down() > topo::kMaxXgmiLinks))
        __builtin_trap();
#elif NETOP_FUZZ_TARGET == 4
    // Wrap the input as the payload of one RTM_NEWLINK message with a consistent header.
    if (size > 1 << 16) return 0;
    std::vector<uint8_t> buf(NLMSG_HDRLEN + size);
    auto* h = reinterpret_cast<nlmsghdr*>(buf.data());
    h->nlmsg_len = uint32_t(buf.size());
    h->nlmsg_type = RTM_NEWLINK;
    std::memcpy(buf.data() + NLMSG_HDRLEN, data, size);
    try {
        (void)nl::parse_link(h);
    } catch (const std::exception&) {
    }
    try {
        (void)nl::parse_link_stats(h);
    } catch (const std::exception&) {
    }
    h->nlmsg_type = RTM_NEWROUTE;  // the same bytes as a route (rtmsg + attributes, RTA_MULTIPATH next hops)
    try {
        (void)nl::parse_route(h);
    } catch (const std::exception&) {
    }
    h->nlmsg_type = RTM_NEWRULE;  // as a FIB rule (fib_rule_hdr + FRA_* attributes)
    try {
        (void)nl::parse_rule(h);
    } catch (const std::exception&) {
    }
    h->nlmsg_type = RTM_NEWADDR;  // as an address (ifaddrmsg + attributes, IPv4 or IPv6)
    try {
        (void)nl::parse_addr(h);
    } catch (const std::exception&) {
    }
    h->nlmsg_type = RTM_GETDCB;  // the same bytes as a DCB netlink reply (dcbmsg + attributes)
    try {
        (void)nl::parse_dcb_u8(h, DCB_ATTR_DCBX);
    } catch (const std::exception&) {
    }
    // The same bytes as an extended-ACK error (nlmsgerr + echoed request + attributes), both with
    // and without the capped echo.
    h->nlmsg_type = NLMSG_ERROR;
    for (uint16_t flags : {uint16_t(NLM_F_ACK_TLVS), uint16_t(NLM_F_ACK_TLVS | NLM_F_CAPPED)}) {
        h->nlmsg_flags = flags;
        (void)nl::ext_ack_msg(h);
    }
#elif NETOP_FUZZ_TARGET == 5
    auto r = arp::parse_reply(data, size);
    if (r) {
        // A reply always carries Ethernet/IPv4 sizes, op 2, and the addresses at their offsets.
        if (size < arp::kPayloadLen || data[7] != 2 || Ipv4::from_net(data + 14) != r->sender_ip) __builtin_trap();
        // The acceptance rule: only a reply from the peer to our own address verifies a NIC.
        if (size >= arp::kPayloadLen + 8) {
            arp::Probe p;
            p.local = Ipv4::from_net(data + arp::kPayloadLen);
            p.peer = Ipv4::from_net(data + arp::kPayloadLen + 4);
            const bool ok = arp::answers(p, *r);
            if (ok != (r->sender_ip == p.peer && r->target_ip == p.local)) __builtin_trap();
            if (ok) {
                arp::record_answer(p, *r, 3000, 1000, 2000);
                if (!p.answered || p.rtt_ns != 1000 || p.verify_ns != 2000 || !(p.peer_mac == r->sender_mac)) __builtin_trap();
            }
        }
    }
    if (size >= 10) {  // requests from arbitrary addresses always encode to a fixed-size payload
        auto req = arp::encode_request(MacAddr::from_bytes(data), Ipv4::from_net(data + 2), Ipv4::from_net(data + 6));
        if (req.size() != arp::kPayloadLen || arp::parse_reply(req.data(), req.size())) __builtin_trap();
    }
#else
#error "define NETOP_FUZZ_TARGET"
#endif
    return 0;
}
