#include "netop/arp.hpp"

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
#include <thread>

namespace netop::arp {

namespace {

constexpr uint16_t kHtypeEthernet = 1;
constexpr uint16_t kOpRequest = 1;
constexpr uint16_t kOpReply = 2;

void put16(uint8_t* p, uint16_t v) {
    p[0] = uint8_t(v >> 8);
    p[1] = uint8_t(v);
}
uint16_t get16(const uint8_t* p) { return uint16_t((p[0] << 8) | p[1]); }

struct Fd {
    int fd = -1;
    ~Fd() {
        if (fd >= 0) ::close(fd);
    }
};

// Only ARP replies reach the socket (offset 0 is the ARP header: SOCK_DGRAM strips Ethernet).
void attach_reply_filter(int fd) {
    static sock_filter code[] = {
        {BPF_LD | BPF_H | BPF_ABS, 0, 0, 6},
        {BPF_JMP | BPF_JEQ | BPF_K, 0, 1, kOpReply},
        {BPF_RET | BPF_K, 0, 0, 0x40000},
        {BPF_RET | BPF_K, 0, 0, 0},
    };
    sock_fprog prog{static_cast<unsigned short>(sizeof code / sizeof code[0]), code};
    if (::setsockopt(fd, SOL_SOCKET, SO_ATTACH_FILTER, &prog, sizeof prog) != 0) throw_errno("SO_ATTACH_FILTER");
}

// Protocol 0 until bind: a socket created for ETH_P_ARP would queue every interface's ARP
// traffic until it is bound to one.
int open_socket(int ifindex) {
    int fd = ::socket(AF_PACKET, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) throw_errno("socket(AF_PACKET, ARP)");
    try {
        attach_reply_filter(fd);
        sockaddr_ll sll{};
        sll.sll_family = AF_PACKET;
        sll.sll_protocol = htons(ETH_P_ARP);
        sll.sll_ifindex = ifindex;
        if (::bind(fd, reinterpret_cast<sockaddr*>(&sll), sizeof sll) != 0) throw_errno("bind(AF_PACKET, ARP)");
    } catch (...) {
        ::close(fd);
        throw;
    }
    return fd;
}

// 0 or the errno of sendto
int send_request(int fd, const Probe& p) {
    auto req = encode_request(p.mac, p.local, p.peer);
    sockaddr_ll to{};
    to.sll_family = AF_PACKET;
    to.sll_protocol = htons(ETH_P_ARP);
    to.sll_ifindex = p.ifindex;
    to.sll_halen = 6;
    std::memset(to.sll_addr, 0xff, 6);
    return ::sendto(fd, req.data(), req.size(), 0, reinterpret_cast<sockaddr*>(&to), sizeof to) < 0 ? errno : 0;
}

}  // namespace

std::vector<uint8_t> encode_request(const MacAddr& sender_mac, Ipv4 sender_ip, Ipv4 target_ip) {
    std::vector<uint8_t> b(kPayloadLen, 0);
    put16(&b[0], kHtypeEthernet);
    put16(&b[2], ETH_P_IP);
    b[4] = 6;
    b[5] = 4;
    put16(&b[6], kOpRequest);
    std::memcpy(&b[8], sender_mac.b.data(), 6);
    sender_ip.to_net(&b[14]);
    // target hardware address: unknown (zero)
    target_ip.to_net(&b[24]);
    return b;
}

std::optional<Reply> parse_reply(const uint8_t* p, size_t n) {
    if (n < kPayloadLen) return std::nullopt;
    if (get16(p) != kHtypeEthernet || get16(p + 2) != ETH_P_IP || p[4] != 6 || p[5] != 4) return std::nullopt;
    if (get16(p + 6) != kOpReply) return std::nullopt;
    Reply r;
    r.sender_mac = MacAddr::from_bytes(p + 8);
    r.sender_ip = Ipv4::from_net(p + 14);
    r.target_ip = Ipv4::from_net(p + 24);
    return r;
}

static void close_concurrently(std::vector<int> fds) {
    std::vector<std::thread> closers;
    for (int fd : fds) {
        try {
            closers.emplace_back([fd] { ::close(fd); });
        } catch (...) {  // no thread: close it here
            ::close(fd);
        }
    }
    for (auto& t : closers) t.join();
}

Prober::~Prober() {
    std::thread t = close_async();
    if (t.joinable()) t.join();
}

std::thread Prober::close_async() {
    if (fds_.empty()) return {};
    std::vector<int> fds;
    for (auto& [idx, fd] : fds_) fds.push_back(fd);
    fds_.clear();
    try {
        return std::thread(close_concurrently, std::move(fds));
    } catch (...) {
        close_concurrently(std::move(fds));
        return {};
    }
}

int Prober::socket_for(int ifindex) {
    auto it = fds_.find(ifindex);
    if (it != fds_.end()) return it->second;
    int fd = open_socket(ifindex);
    fds_[ifindex] = fd;
    return fd;
}

bool answers(const Probe& p, const Reply& r) { return r.sender_ip == p.peer && r.target_ip == p.local; }

void record_answer(Probe& p, const Reply& r, int64_t now, int64_t first_sent, int64_t last_sent) {
    p.answered = true;
    p.peer_mac = r.sender_mac;
    p.verify_ns = first_sent ? now - first_sent : 0;
    p.rtt_ns = last_sent ? now - last_sent : p.verify_ns;
}

bool Prober::probe(std::vector<Probe>& probes, int64_t timeout_ns, int64_t retry_ns, int stop_fd) {
    Fd ep{::epoll_create1(EPOLL_CLOEXEC)};
    if (ep.fd < 0) throw_errno("epoll_create1");
    if (stop_fd >= 0) {
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.u64 = ~uint64_t(0);
        if (::epoll_ctl(ep.fd, EPOLL_CTL_ADD, stop_fd, &ev) != 0) throw_errno("epoll_ctl(stop)");
    }
    uint8_t buf[256];
    const int64_t t0 = mono_ns();
    std::vector<int> fds(probes.size(), -1);
    std::vector<int64_t> first_sent(probes.size(), 0), last_sent(probes.size(), 0);
    for (size_t i = 0; i < probes.size(); ++i) {
        Probe& p = probes[i];
        p.answered = false;
        p.requests = 0;
        p.error.clear();
        try {
            fds[i] = socket_for(p.ifindex);
            while (::recv(fds[i], buf, sizeof buf, MSG_DONTWAIT) >= 0) {
            }  // replies to an earlier probe do not answer this one
            epoll_event ev{};
            ev.events = EPOLLIN;
            ev.data.u64 = i;
            if (::epoll_ctl(ep.fd, EPOLL_CTL_ADD, fds[i], &ev) != 0) throw_errno("epoll_ctl(ARP)");
        } catch (const std::exception& e) {
            p.error = e.what();
        }
    }
    const int64_t deadline = t0 + timeout_ns;
    int64_t next_send = t0;
    auto pending = [&] {
        return std::any_of(probes.begin(), probes.end(), [](const Probe& p) { return !p.answered && p.error.empty(); });
    };
    while (pending()) {
        int64_t now = mono_ns();
        if (now >= deadline) break;
        if (now >= next_send) {
            for (size_t i = 0; i < probes.size(); ++i) {
                Probe& p = probes[i];
                if (p.answered || !p.error.empty()) continue;
                const int err = send_request(fds[i], p);
                if (err == 0) {
                    last_sent[i] = mono_ns();
                    if (p.requests++ == 0) first_sent[i] = last_sent[i];
                } else if (err != ENETDOWN && err != ENXIO && err != ENOBUFS && err != EAGAIN) {
                    // (a link that is down may come back within the timeout: those retry)
                    p.error = "sendto(ARP) " + p.ifname + ": " + std::strerror(err);
                }
            }
            next_send = now + retry_ns;
        }
        const int64_t until = std::min(deadline, next_send);
        int ms = int(std::max<int64_t>(0, (until - mono_ns() + 999999) / 1000000));
        epoll_event evs[16];
        int k = ::epoll_wait(ep.fd, evs, 16, ms);
        if (k < 0) {
            if (errno == EINTR) continue;
            throw_errno("epoll_wait(ARP)");
        }
        for (int e = 0; e < k; ++e) {
            if (evs[e].data.u64 == ~uint64_t(0)) return false;
            size_t i = size_t(evs[e].data.u64);
            Probe& p = probes[i];
            for (;;) {
                ssize_t n = ::recv(fds[i], buf, sizeof buf, MSG_DONTWAIT);
                if (n < 0) break;  // EAGAIN: drained
                auto r = parse_reply(buf, size_t(n));
                if (!r || p.answered || !answers(p, *r)) continue;
                record_answer(p, *r, mono_ns(), first_sent[i] ? first_sent[i] : t0, last_sent[i]);
            }
        }
    }
    return true;
}

bool probe_all(std::vector<Probe>& probes, int64_t timeout_ns, int64_t retry_ns, int stop_fd) {
    Prober p;
    return p.probe(probes, timeout_ns, retry_ns, stop_fd);
}

}  // namespace netop::arp
