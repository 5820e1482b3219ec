// Common value types for the MI355X network agent: MAC / IPv4 / prefix, errors, helpers.
//
// Parity notes: the reference keeps addresses as Go net.IP / net.HardwareAddr
// (reference cmd/discover/network.go:65-74).  Here everything on the hot path is a
// fixed-size value type (uint32 IPv4 in host order, 6-byte MAC) so LLDP decode ->
// address derivation -> netlink request never allocates.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <optional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <system_error>
#include <vector>

namespace netop {

struct MacAddr {
    std::array<uint8_t, 6> b{};

    static std::optional<MacAddr> parse(std::string_view s);
    static MacAddr from_bytes(const uint8_t* p) {
        MacAddr m;
        std::memcpy(m.b.data(), p, 6);
        return m;
    }
    std::string str() const;  // lower-case "aa:bb:cc:dd:ee:ff" (Go net.HardwareAddr.String())
    bool is_zero() const {
        for (auto x : b)
            if (x) return false;
        return true;
    }
    bool operator==(const MacAddr& o) const { return b == o.b; }
    bool operator!=(const MacAddr& o) const { return b != o.b; }
};

// IPv4 address, host byte order.
struct Ipv4 {
    uint32_t v = 0;

    static std::optional<Ipv4> parse(std::string_view s);
    static Ipv4 from_net(const void* p) {  // 4 bytes network order
        const auto* q = static_cast<const uint8_t*>(p);
        return Ipv4{(uint32_t(q[0]) << 24) | (uint32_t(q[1]) << 16) | (uint32_t(q[2]) << 8) | q[3]};
    }
    void to_net(void* p) const {
        auto* q = static_cast<uint8_t*>(p);
        q[0] = uint8_t(v >> 24);
        q[1] = uint8_t(v >> 16);
        q[2] = uint8_t(v >> 8);
        q[3] = uint8_t(v);
    }
    std::string str() const;
    bool operator==(const Ipv4& o) const { return v == o.v; }
    bool operator!=(const Ipv4& o) const { return v != o.v; }
    bool operator<(const Ipv4& o) const { return v < o.v; }
};

inline uint32_t prefix_mask(int len) { return len <= 0 ? 0u : (len >= 32 ? 0xffffffffu : ~((1u << (32 - len)) - 1)); }

struct Ipv4Prefix {
    Ipv4 addr;
    int len = 32;

    // Parses "a.b.c.d/len" (strict, like Go net.ParseCIDR for IPv4).
    static std::optional<Ipv4Prefix> parse(std::string_view s);
    Ipv4 mask() const { return Ipv4{prefix_mask(len)}; }
    Ipv4 network() const { return Ipv4{addr.v & prefix_mask(len)}; }
    Ipv4Prefix masked() const { return Ipv4Prefix{network(), len}; }
    std::string str() const { return addr.str() + "/" + std::to_string(len); }
    bool contains(Ipv4 a) const { return (a.v & prefix_mask(len)) == network().v; }
    bool operator==(const Ipv4Prefix& o) const { return addr == o.addr && len == o.len; }
};

// Error carrying an errno (netlink / syscalls).  code()==EEXIST etc. is checked by callers.
class SysError : public std::runtime_error {
   public:
    SysError(int err, const std::string& what);
    int code() const { return err_; }

   private:
    int err_;
};

[[noreturn]] void throw_errno(const std::string& what);

// printf-style std::string formatting.
std::string strfmt(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

std::vector<std::string> split(std::string_view s, char sep);           // Go strings.Split semantics
std::vector<std::string> split_ws(std::string_view s);                   // Go strings.Fields semantics
std::string trim(std::string_view s);
std::string to_upper(std::string_view s);
std::string join(const std::vector<std::string>& v, std::string_view sep);

// Monotonic clock in nanoseconds.
int64_t mono_ns();
// Wall clock (CLOCK_REALTIME) in nanoseconds.
int64_t wall_ns();

// Parses a Go time.Duration string ("90s", "1m30s", "250ms", "1.5h", "0").  Returns nanoseconds.
std::optional<int64_t> parse_go_duration(std::string_view s);
std::string format_go_duration(int64_t ns);

// Read a whole small file (sysfs / procfs).  nullopt if unreadable.
std::optional<std::string> read_file(const std::string& path);
// Atomically replace `path` (write temp + fsync + rename) with given permission bits.
void write_file_atomic(const std::string& path, std::string_view content, unsigned mode = 0644);
// Whether write_file_atomic fsyncs before the rename (default off: every artifact is rewritten
// from scratch whenever the agent starts, so durability buys nothing, and fsync costs ~0.2 ms
// per file on the critical path; the rename alone keeps readers from seeing partial files).
void set_durable_writes(bool on);
bool path_exists(const std::string& path);
bool is_dir(const std::string& path);
void mkdir_p(const std::string& path, unsigned mode = 0755);
std::string path_join(std::string_view a, std::string_view b);
std::string path_dirname(std::string_view p);
std::string path_basename(std::string_view p);
std::optional<std::string> realpath_of(const std::string& p);
std::vector<std::string> list_dir(const std::string& dir);  // sorted entry names, no . / ..

}  // namespace netop
