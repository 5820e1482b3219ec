// AF_PACKET LLDP receive / transmit.
//
// Replaces the reference's gopacket+libpcap receiver (reference pkg/lldp/client.go:73-149),
// which opened one promiscuous pcap handle per NIC (5 s read timeout) inside one
// goroutine per NIC and then waited on a barrier for all of them
// (cmd/discover/main.go:84-122).  Here:
//   * one non-blocking AF_PACKET socket per NIC, a hand-written classic-BPF filter
//     (EtherType 0x88cc, optionally behind one 802.1Q tag) attached before bind so no
//     unfiltered frame is ever queued;
//   * LLDP multicast group membership instead of full promiscuous mode (promisc is
//     still available for parity);
//   * a single epoll loop over every NIC; each frame is handed to the caller the moment
//     it arrives, so configuration is pipelined per NIC rather than barrier-synchronised.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "netop/common.hpp"
#include "netop/lldp.hpp"

namespace netop::pkt {

struct ListenerStats {
    uint64_t frames = 0;     // LLDP frames accepted
    uint64_t own = 0;        // frames sourced from our own MAC (ignored, client.go:108-111)
    uint64_t malformed = 0;  // frames that failed to decode
    uint64_t wakeups = 0;    // epoll wakeups
};

class LldpSocket {
   public:
    LldpSocket(const std::string& ifname, int ifindex, const MacAddr& own_mac, bool promisc);
    ~LldpSocket();
    LldpSocket(const LldpSocket&) = delete;
    LldpSocket& operator=(const LldpSocket&) = delete;

    int fd() const { return fd_; }
    int release_fd() {  // the caller closes it
        int f = fd_;
        fd_ = -1;
        return f;
    }
    const std::string& ifname() const { return ifname_; }
    int ifindex() const { return ifindex_; }
    const MacAddr& own_mac() const { return own_; }
    const ListenerStats& stats() const { return stats_; }  // this socket's share

    // Reads every queued frame without blocking; returns the decoded LLDPDUs that
    // did not come from our own MAC.
    std::vector<lldp::Frame> drain(ListenerStats* stats);
    void send(const std::vector<uint8_t>& frame);

   private:
    int fd_ = -1;
    std::string ifname_;
    int ifindex_ = 0;
    MacAddr own_;
    ListenerStats stats_;
};

enum class ListenResult { Stopped, Deadline, Interrupted };

class LldpListener {
   public:
    LldpListener();
    ~LldpListener();
    void add(const std::string& ifname, int ifindex, const MacAddr& own_mac, bool promisc);
    void remove(const std::string& ifname);
    // Transmits a frame on a listened interface; false if the interface is unknown.
    bool send(const std::string& ifname, const std::vector<uint8_t>& frame);
    size_t size() const { return socks_.size(); }

    // Runs until `on_frame` returns true (stop), the absolute CLOCK_MONOTONIC deadline
    // passes, or `interrupt_fd` (e.g. a signalfd; -1 = none) becomes readable.
    ListenResult run(int64_t deadline_mono_ns,
                     const std::function<bool(const std::string& ifname, const lldp::Frame& frame)>& on_frame,
                     int interrupt_fd = -1);
    const ListenerStats& stats() const { return stats_; }
    // One interface's counters (a default-constructed record for an unknown one).
    ListenerStats stats_for(const std::string& ifname) const;

   private:
    int epfd_ = -1;
    std::vector<std::unique_ptr<LldpSocket>> socks_;
    ListenerStats stats_;
};

// Attach the LLDP classic-BPF program to any packet socket (exposed for tests).
void attach_lldp_filter(int fd);

}  // namespace netop::pkt
