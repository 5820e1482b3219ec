#include "netop/packet.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <linux/filter.h>
#include <linux/if_ether.h>
#include <linux/if_packet.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <system_error>
#include <thread>

#include "netop/log.hpp"

#ifndef PACKET_IGNORE_OUTGOING
#define PACKET_IGNORE_OUTGOING 23
#endif

namespace netop::pkt {

void attach_lldp_filter(int fd) {
    // Accept EtherType 0x88cc, or 0x8100 + inner 0x88cc; drop everything else.
    static sock_filter code[] = {
        {BPF_LD | BPF_H | BPF_ABS, 0, 0, 12},
        {BPF_JMP | BPF_JEQ | BPF_K, 3, 0, lldp::kEtherType},
        {BPF_JMP | BPF_JEQ | BPF_K, 0, 3, 0x8100},
        {BPF_LD | BPF_H | BPF_ABS, 0, 0, 16},
        {BPF_JMP | BPF_JEQ | BPF_K, 0, 1, lldp::kEtherType},
        {BPF_RET | BPF_K, 0, 0, 0x40000},
        {BPF_RET | BPF_K, 0, 0, 0},
    };
    sock_fprog prog{static_cast<unsigned short>(sizeof code / sizeof code[0]), code};
    if (::setsockopt(fd, SOL_SOCKET, SO_ATTACH_FILTER, &prog, sizeof prog) != 0) throw_errno("SO_ATTACH_FILTER");
}

LldpSocket::LldpSocket(const std::string& ifname, int ifindex, const MacAddr& own_mac, bool promisc)
    : ifname_(ifname), ifindex_(ifindex), own_(own_mac) {
    // Protocol 0: nothing is queued until bind(), so the filter is in place first.
    fd_ = ::socket(AF_PACKET, SOCK_RAW | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd_ < 0) throw_errno("socket(AF_PACKET) for " + ifname);
    try {
        attach_lldp_filter(fd_);
        int one = 1;
        ::setsockopt(fd_, SOL_PACKET, PACKET_IGNORE_OUTGOING, &one, sizeof one);  // best effort (>= 4.20)
        sockaddr_ll sll{};
        sll.sll_family = AF_PACKET;
        sll.sll_protocol = htons(ETH_P_ALL);
        sll.sll_ifindex = ifindex;
        if (::bind(fd_, reinterpret_cast<sockaddr*>(&sll), sizeof sll) != 0) throw_errno("bind(AF_PACKET) " + ifname);
        for (const MacAddr* g : {&lldp::kNearestBridge, &lldp::kNearestNonTpmrBridge, &lldp::kNearestCustomerBridge}) {
            packet_mreq mr{};
            mr.mr_ifindex = ifindex;
            mr.mr_type = PACKET_MR_MULTICAST;
            mr.mr_alen = 6;
            std::memcpy(mr.mr_address, g->b.data(), 6);
            if (::setsockopt(fd_, SOL_PACKET, PACKET_ADD_MEMBERSHIP, &mr, sizeof mr) != 0)
                NLOG_V(2, "PACKET_ADD_MEMBERSHIP %s on %s: %s", g->str().c_str(), ifname.c_str(), std::strerror(errno));
        }
        if (promisc) {
            packet_mreq mr{};
            mr.mr_ifindex = ifindex;
            mr.mr_type = PACKET_MR_PROMISC;
            if (::setsockopt(fd_, SOL_PACKET, PACKET_ADD_MEMBERSHIP, &mr, sizeof mr) != 0)
                throw_errno("PACKET_MR_PROMISC on " + ifname);
        }
    } catch (...) {
        ::close(fd_);
        fd_ = -1;
        throw;
    }
}

LldpSocket::~LldpSocket() {
    if (fd_ >= 0) ::close(fd_);  // memberships / promisc are dropped with the socket
}

std::vector<lldp::Frame> LldpSocket::drain(ListenerStats* stats) {
    std::vector<lldp::Frame> out;
    alignas(8) uint8_t buf[9216 + 64];
    for (;;) {
        sockaddr_ll from{};
        socklen_t fl = sizeof from;
        ssize_t n = ::recvfrom(fd_, buf, sizeof buf, MSG_DONTWAIT, reinterpret_cast<sockaddr*>(&from), &fl);
        if (n < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            if (errno == ENETDOWN) break;  // link went down under us; keep the socket
            throw_errno("recvfrom(AF_PACKET) " + ifname_);
        }
        if (from.sll_pkttype == PACKET_OUTGOING) continue;
        if (n >= 12 && std::memcmp(buf + 6, own_.b.data(), 6) == 0) {
            ++stats_.own;
            if (stats) ++stats->own;
            continue;
        }
        lldp::DecodeError err;
        auto f = lldp::decode(buf, size_t(n), &err);
        if (!f) {
            ++stats_.malformed;
            if (stats) ++stats->malformed;
            NLOG_V(4, "%s: dropping malformed LLDP frame (%zd bytes): %s", ifname_.c_str(), n, lldp::to_string(err));
            continue;
        }
        ++stats_.frames;
        if (stats) ++stats->frames;
        out.push_back(std::move(*f));
    }
    return out;
}

void LldpSocket::send(const std::vector<uint8_t>& frame) {
    if (frame.size() < 14) throw SysError(EINVAL, "frame too short");
    sockaddr_ll sll{};
    sll.sll_family = AF_PACKET;
    sll.sll_ifindex = ifindex_;
    sll.sll_halen = 6;
    std::memcpy(sll.sll_addr, frame.data(), 6);
    for (;;) {
        ssize_t n = ::sendto(fd_, frame.data(), frame.size(), 0, reinterpret_cast<sockaddr*>(&sll), sizeof sll);
        if (n >= 0) return;
        if (errno == EINTR) continue;
        throw_errno("sendto(AF_PACKET) " + ifname_);
    }
}

LldpListener::LldpListener() {
    epfd_ = ::epoll_create1(EPOLL_CLOEXEC);
    if (epfd_ < 0) throw_errno("epoll_create1");
}

LldpListener::~LldpListener() {
    // Closing a packet socket waits for an RCU grace period (packet_release -> synchronize_net),
    // ~15-20 ms each: one after the other, 8 NICs held SIGTERM -> exit at ~140 ms (the rolling
    // update of the DaemonSet waits for that).  Closed concurrently, the waits overlap.
    std::vector<std::thread> closers;
    for (auto& s : socks_) {
        if (!s) continue;
        try {
            closers.emplace_back([p = s.get()] { ::close(p->release_fd()); });
        } catch (...) {  // no thread (destructors must not throw): close it here
            ::close(s->release_fd());
        }
    }
    for (auto& t : closers) t.join();
    socks_.clear();
    if (epfd_ >= 0) ::close(epfd_);
}

void LldpListener::add(const std::string& ifname, int ifindex, const MacAddr& own_mac, bool promisc) {
    auto s = std::make_unique<LldpSocket>(ifname, ifindex, own_mac, promisc);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = uint64_t(socks_.size());
    if (::epoll_ctl(epfd_, EPOLL_CTL_ADD, s->fd(), &ev) != 0) throw_errno("epoll_ctl ADD " + ifname);
    socks_.push_back(std::move(s));
}

void LldpListener::remove(const std::string& ifname) {
    for (auto& s : socks_) {
        if (s && s->ifname() == ifname) {
            ::epoll_ctl(epfd_, EPOLL_CTL_DEL, s->fd(), nullptr);
            s.reset();  // keep slot indices stable for epoll data
        }
    }
}

ListenerStats LldpListener::stats_for(const std::string& ifname) const {
    for (auto& s : socks_)
        if (s && s->ifname() == ifname) return s->stats();
    return {};
}

bool LldpListener::send(const std::string& ifname, const std::vector<uint8_t>& frame) {
    for (auto& s : socks_) {
        if (s && s->ifname() == ifname) {
            s->send(frame);
            return true;
        }
    }
    return false;
}

ListenResult LldpListener::run(int64_t deadline,
                               const std::function<bool(const std::string&, const lldp::Frame&)>& on_frame,
                               int interrupt_fd) {
    constexpr uint64_t kInterruptTag = ~uint64_t(0);
    if (interrupt_fd >= 0) {
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.u64 = kInterruptTag;
        if (::epoll_ctl(epfd_, EPOLL_CTL_ADD, interrupt_fd, &ev) != 0 && errno != EEXIST)
            throw_errno("epoll_ctl ADD interrupt fd");
    }
    struct Cleanup {
        int ep, fd;
        ~Cleanup() {
            if (fd >= 0) ::epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
        }
    } cleanup{epfd_, interrupt_fd};

    // Frames may already be queued (they arrived between bind and run): drain first.
    for (auto& s : socks_) {
        if (!s) continue;
        for (auto& f : s->drain(&stats_))
            if (on_frame(s->ifname(), f)) return ListenResult::Stopped;
    }
    epoll_event evs[64];
    for (;;) {
        int64_t now = mono_ns();
        if (now >= deadline) return ListenResult::Deadline;
        int timeout_ms = int(std::min<int64_t>((deadline - now + 999999) / 1000000, 1 << 30));
        int n = ::epoll_wait(epfd_, evs, 64, timeout_ms);
        if (n < 0) {
            if (errno == EINTR) continue;
            throw_errno("epoll_wait");
        }
        ++stats_.wakeups;
        for (int i = 0; i < n; ++i) {
            if (evs[i].data.u64 == kInterruptTag) return ListenResult::Interrupted;
            auto idx = size_t(evs[i].data.u64);
            if (idx >= socks_.size() || !socks_[idx]) continue;
            auto& s = socks_[idx];
            std::string name = s->ifname();
            for (auto& f : s->drain(&stats_))
                if (on_frame(name, f)) return ListenResult::Stopped;
        }
    }
}

}  // namespace netop::pkt
