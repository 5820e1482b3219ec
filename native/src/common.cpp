#include "netop/common.hpp"

#include <atomic>

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

namespace netop {

static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

std::optional<MacAddr> MacAddr::parse(std::string_view s) {
    // Accept "aa:bb:cc:dd:ee:ff" and "aa-bb-cc-dd-ee-ff".
    if (s.size() != 17) return std::nullopt;
    MacAddr m;
    for (int i = 0; i < 6; ++i) {
        int h = hexval(s[i * 3]), l = hexval(s[i * 3 + 1]);
        if (h < 0 || l < 0) return std::nullopt;
        if (i < 5 && s[i * 3 + 2] != ':' && s[i * 3 + 2] != '-') return std::nullopt;
        m.b[i] = uint8_t(h << 4 | l);
    }
    return m;
}

std::string MacAddr::str() const {
    char buf[18];
    std::snprintf(buf, sizeof buf, "%02x:%02x:%02x:%02x:%02x:%02x", b[0], b[1], b[2], b[3], b[4], b[5]);
    return buf;
}

std::optional<Ipv4> Ipv4::parse(std::string_view s) {
    uint32_t v = 0;
    size_t i = 0;
    for (int part = 0; part < 4; ++part) {
        if (i >= s.size() || s[i] < '0' || s[i] > '9') return std::nullopt;
        size_t start = i;
        uint32_t x = 0;
        while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
            x = x * 10 + uint32_t(s[i] - '0');
            if (x > 255 || i - start >= 3) return std::nullopt;
            ++i;
        }
        if (i - start > 1 && s[start] == '0') return std::nullopt;  // Go rejects leading zeros
        v = (v << 8) | x;
        if (part < 3) {
            if (i >= s.size() || s[i] != '.') return std::nullopt;
            ++i;
        }
    }
    if (i != s.size()) return std::nullopt;
    return Ipv4{v};
}

std::string Ipv4::str() const {
    char buf[16];
    std::snprintf(buf, sizeof buf, "%u.%u.%u.%u", v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255);
    return buf;
}

std::optional<Ipv4Prefix> Ipv4Prefix::parse(std::string_view s) {
    auto slash = s.find('/');
    if (slash == std::string_view::npos) return std::nullopt;
    auto a = Ipv4::parse(s.substr(0, slash));
    if (!a) return std::nullopt;
    auto ls = s.substr(slash + 1);
    if (ls.empty() || ls.size() > 2) return std::nullopt;
    int len = 0;
    for (char c : ls) {
        if (c < '0' || c > '9') return std::nullopt;
        len = len * 10 + (c - '0');
    }
    if (ls.size() > 1 && ls[0] == '0') return std::nullopt;
    if (len > 32) return std::nullopt;
    return Ipv4Prefix{*a, len};
}

SysError::SysError(int err, const std::string& what)
    : std::runtime_error(what + ": " + std::strerror(err)), err_(err) {}

void throw_errno(const std::string& what) { throw SysError(errno, what); }

std::string strfmt(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    char small[256];
    va_list ap2;
    va_copy(ap2, ap);
    int n = std::vsnprintf(small, sizeof small, fmt, ap);
    va_end(ap);
    if (n < 0) {
        va_end(ap2);
        return {};
    }
    if (size_t(n) < sizeof small) {
        va_end(ap2);
        return std::string(small, size_t(n));
    }
    std::string out(size_t(n), '\0');
    std::vsnprintf(out.data(), size_t(n) + 1, fmt, ap2);
    va_end(ap2);
    return out;
}

std::vector<std::string> split(std::string_view s, char sep) {
    std::vector<std::string> out;
    size_t start = 0;
    for (;;) {
        size_t p = s.find(sep, start);
        if (p == std::string_view::npos) {
            out.emplace_back(s.substr(start));
            return out;
        }
        out.emplace_back(s.substr(start, p - start));
        start = p + 1;
    }
}

static bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

std::vector<std::string> split_ws(std::string_view s) {
    std::vector<std::string> out;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && is_space(s[i])) ++i;
        size_t start = i;
        while (i < s.size() && !is_space(s[i])) ++i;
        if (i > start) out.emplace_back(s.substr(start, i - start));
    }
    return out;
}

std::string trim(std::string_view s) {
    size_t a = 0, b = s.size();
    while (a < b && is_space(s[a])) ++a;
    while (b > a && is_space(s[b - 1])) --b;
    return std::string(s.substr(a, b - a));
}

std::string to_upper(std::string_view s) {
    std::string o(s);
    for (auto& c : o)
        if (c >= 'a' && c <= 'z') c = char(c - 'a' + 'A');
    return o;
}

std::string join(const std::vector<std::string>& v, std::string_view sep) {
    std::string o;
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) o += sep;
        o += v[i];
    }
    return o;
}

int64_t mono_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return int64_t(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

int64_t wall_ns() {
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return int64_t(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

std::optional<int64_t> parse_go_duration(std::string_view s) {
    // Grammar of Go time.ParseDuration: [-+]? ( number unit )+ | "0"
    if (s.empty()) return std::nullopt;
    bool neg = false;
    if (s[0] == '-' || s[0] == '+') {
        neg = s[0] == '-';
        s.remove_prefix(1);
    }
    if (s == "0") return 0;
    if (s.empty()) return std::nullopt;
    long double total = 0;
    while (!s.empty()) {
        size_t i = 0;
        bool digits = false;
        long double num = 0;
        while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
            num = num * 10 + (s[i] - '0');
            ++i;
            digits = true;
        }
        if (i < s.size() && s[i] == '.') {
            ++i;
            long double scale = 0.1L;
            while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
                num += (s[i] - '0') * scale;
                scale /= 10;
                ++i;
                digits = true;
            }
        }
        if (!digits) return std::nullopt;
        size_t u = i;
        while (u < s.size() && !(s[u] >= '0' && s[u] <= '9') && s[u] != '.') ++u;
        auto unit = s.substr(i, u - i);
        long double mult;
        if (unit == "ns")
            mult = 1;
        else if (unit == "us" || unit == "\xc2\xb5s" || unit == "\xce\xbcs")
            mult = 1e3L;
        else if (unit == "ms")
            mult = 1e6L;
        else if (unit == "s")
            mult = 1e9L;
        else if (unit == "m")
            mult = 60e9L;
        else if (unit == "h")
            mult = 3600e9L;
        else
            return std::nullopt;  // missing or unknown unit
        total += num * mult;
        s.remove_prefix(u);
    }
    if (total > 9.2e18L) return std::nullopt;
    int64_t ns = int64_t(std::llround(double(total)));
    return neg ? -ns : ns;
}

std::string format_go_duration(int64_t ns) {
    if (ns == 0) return "0s";
    std::string sign = ns < 0 ? "-" : "";
    uint64_t u = uint64_t(ns < 0 ? -ns : ns);
    if (u < 1000000000ULL) {
        if (u < 1000) return sign + std::to_string(u) + "ns";
        if (u < 1000000) return sign + strfmt("%gus", double(u) / 1e3);
        return sign + strfmt("%gms", double(u) / 1e6);
    }
    uint64_t h = u / 3600000000000ULL;
    u %= 3600000000000ULL;
    uint64_t m = u / 60000000000ULL;
    u %= 60000000000ULL;
    std::string out = sign;
    if (h) out += std::to_string(h) + "h";
    if (h || m) out += std::to_string(m) + "m";
    out += strfmt("%gs", double(u) / 1e9);
    return out;
}

std::optional<std::string> read_file(const std::string& path) {
    int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return std::nullopt;
    std::string out;
    char buf[4096];
    for (;;) {
        ssize_t n = ::read(fd, buf, sizeof buf);
        if (n < 0) {
            if (errno == EINTR) continue;
            ::close(fd);
            return std::nullopt;
        }
        if (n == 0) break;
        out.append(buf, size_t(n));
    }
    ::close(fd);
    return out;
}

static std::atomic<bool> g_durable_writes{false};

void set_durable_writes(bool on) { g_durable_writes.store(on, std::memory_order_relaxed); }

void write_file_atomic(const std::string& path, std::string_view content, unsigned mode) {
    std::string tmp = path + ".tmp." + std::to_string(::getpid());
    int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, mode);
    if (fd < 0) throw_errno("open " + tmp);
    size_t off = 0;
    while (off < content.size()) {
        ssize_t n = ::write(fd, content.data() + off, content.size() - off);
        if (n < 0) {
            if (errno == EINTR) continue;
            int e = errno;
            ::close(fd);
            ::unlink(tmp.c_str());
            throw SysError(e, "write " + tmp);
        }
        off += size_t(n);
    }
    ::fchmod(fd, mode);  // umask-independent, like Go os.WriteFile on a new file with 0644
    if (g_durable_writes.load(std::memory_order_relaxed)) ::fsync(fd);
    ::close(fd);
    if (::rename(tmp.c_str(), path.c_str()) != 0) {
        int e = errno;
        ::unlink(tmp.c_str());
        throw SysError(e, "rename " + tmp + " -> " + path);
    }
}

bool path_exists(const std::string& path) {
    struct stat st;
    return ::stat(path.c_str(), &st) == 0;
}

bool is_dir(const std::string& path) {
    struct stat st;
    return ::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

void mkdir_p(const std::string& path, unsigned mode) {
    if (path.empty()) return;
    std::string cur;
    for (auto& part : split(path, '/')) {
        if (part.empty()) {
            if (cur.empty()) cur = "/";
            continue;
        }
        if (!cur.empty() && cur.back() != '/') cur += '/';
        cur += part;
        if (::mkdir(cur.c_str(), mode) != 0 && errno != EEXIST) throw_errno("mkdir " + cur);
    }
    if (!is_dir(path)) throw SysError(ENOTDIR, "mkdir " + path);
}

std::string path_join(std::string_view a, std::string_view b) {
    if (a.empty()) return std::string(b);
    if (b.empty()) return std::string(a);
    std::string o(a);
    if (o.back() == '/' && b.front() == '/')
        o.pop_back();
    else if (o.back() != '/' && b.front() != '/')
        o += '/';
    o += b;
    return o;
}

std::string path_dirname(std::string_view p) {
    while (p.size() > 1 && p.back() == '/') p.remove_suffix(1);
    auto s = p.rfind('/');
    if (s == std::string_view::npos) return ".";
    if (s == 0) return "/";
    return std::string(p.substr(0, s));
}

std::string path_basename(std::string_view p) {
    while (p.size() > 1 && p.back() == '/') p.remove_suffix(1);
    auto s = p.rfind('/');
    return std::string(s == std::string_view::npos ? p : p.substr(s + 1));
}

std::optional<std::string> realpath_of(const std::string& p) {
    char* r = ::realpath(p.c_str(), nullptr);
    if (!r) return std::nullopt;
    std::string out(r);
    std::free(r);
    return out;
}

std::vector<std::string> list_dir(const std::string& dir) {
    std::vector<std::string> out;
    DIR* d = ::opendir(dir.c_str());
    if (!d) return out;
    while (auto* e = ::readdir(d)) {
        if (!std::strcmp(e->d_name, ".") || !std::strcmp(e->d_name, "..")) continue;
        out.emplace_back(e->d_name);
    }
    ::closedir(d);
    std::sort(out.begin(), out.end());
    return out;
}

}  // namespace netop
