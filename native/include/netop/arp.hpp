// Peer reachability over ARP (RFC 826), for `discover --verify-peers`.
//
// LLDP proves that a switch port is attached and tells the agent its /30; it does not prove
// that the port answers on that /30.  A switch port whose Port Description was edited but whose
// interface address was not (or the reverse) gives a node that is labelled ready and whose RCCL
// traffic goes nowhere.  The reference has no such check (the label follows
// the address configuration).  Here every configured NIC asks its switch-side /30 address
// "who-has" from its own address, all NICs at once on one epoll, and the agent counts a NIC as
// configured only once the peer has answered.
//
// One SOCK_DGRAM AF_PACKET socket per NIC bound to ETH_P_ARP on that ifindex: the kernel adds
// and strips the Ethernet header, so the code deals in the 28-byte ARP payload only.
#pragma once

#include <cstdint>
#include <map>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "netop/common.hpp"

namespace netop::arp {

constexpr size_t kPayloadLen = 28;  // Ethernet/IPv4 ARP: htype, ptype, hlen, plen, op, sha, spa, tha, tpa

// The who-has request `sender_ip` (at `sender_mac`) asks about `target_ip`.
std::vector<uint8_t> encode_request(const MacAddr& sender_mac, Ipv4 sender_ip, Ipv4 target_ip);

struct Reply {
    MacAddr sender_mac;
    Ipv4 sender_ip;
    Ipv4 target_ip;
};

// A reply (op 2) for Ethernet/IPv4; nullopt for anything else (requests, other hardware,
// truncated payloads).
std::optional<Reply> parse_reply(const uint8_t* p, size_t n);

struct Probe {
    std::string ifname;
    int ifindex = 0;
    MacAddr mac;     // the NIC's
    Ipv4 local;      // our /30 address
    Ipv4 peer;       // the switch-side /30 address that must answer
    // results
    bool answered = false;
    int64_t rtt_ns = 0;     // round trip: the last request sent before the answer, to the answer
    int64_t verify_ns = 0;  // time to verify: the first request to the answer (retries included)
    MacAddr peer_mac;
    int requests = 0;
    std::string error;  // socket errors; empty when the peer just stayed silent
};

// Keeps one socket per interface open across probes.  Closing a packet socket waits for an RCU
// grace period (packet_release -> synchronize_net, 10-20 ms), so the agent does not close them
// on its way to readiness: they live as long as the prober, are reused by the monitor, and are
// closed concurrently at the end (close_async overlaps that wait with the LLDP sockets').
class Prober {
   public:
    Prober() = default;
    ~Prober();
    Prober(const Prober&) = delete;
    Prober& operator=(const Prober&) = delete;

    // Probes every entry at once: a request right away and again every `retry_ns` until the
    // peer answers, `timeout_ns` passes, or `stop_fd` (-1 = none) becomes readable.  Returns
    // false when interrupted by `stop_fd`.
    bool probe(std::vector<Probe>& probes, int64_t timeout_ns, int64_t retry_ns, int stop_fd = -1);
    // Starts closing every socket (one thread per socket); join the result before exiting.
    std::thread close_async();
    size_t sockets() const { return fds_.size(); }

   private:
    int socket_for(int ifindex);
    std::map<int, int> fds_;  // ifindex -> fd
};

// Whether `r` answers probe `p`: a reply from the peer's address *to our own* address.  A reply
// aimed at another local address (another NIC on the segment, a stale exchange) or a gratuitous
// one (target = sender) does not verify that this NIC's /30 works.
bool answers(const Probe& p, const Reply& r);
// Records an accepted reply at `now` (both times from the requests' send times).
void record_answer(Probe& p, const Reply& r, int64_t now, int64_t first_sent, int64_t last_sent);

// One-shot: a Prober for one call (its sockets are closed before returning).
bool probe_all(std::vector<Probe>& probes, int64_t timeout_ns, int64_t retry_ns, int stop_fd = -1);

}  // namespace netop::arp
