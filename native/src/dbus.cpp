#include "netop/dbus.hpp"

#include <errno.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "netop/common.hpp"

namespace netop::dbus {

// ---------------------------------------------------------------------------
// Value accessors
// ---------------------------------------------------------------------------
const std::string& Value::as_string() const {
    if (auto* p = std::get_if<std::string>(&v)) return *p;
    throw std::runtime_error("dbus value is not a string (sig " + sig + ")");
}
bool Value::as_bool() const {
    if (auto* p = std::get_if<bool>(&v)) return *p;
    throw std::runtime_error("dbus value is not a boolean (sig " + sig + ")");
}
uint32_t Value::as_u32() const {
    if (auto* p = std::get_if<uint32_t>(&v)) return *p;
    throw std::runtime_error("dbus value is not a uint32 (sig " + sig + ")");
}
const Array& Value::as_array() const {
    if (auto* p = std::get_if<std::shared_ptr<Array>>(&v)) return **p;
    throw std::runtime_error("dbus value is not a container (sig " + sig + ")");
}
const Value& Value::variant_inner() const {
    const auto& a = as_array();
    if (sig != "v" || a.size() != 1) throw std::runtime_error("dbus value is not a variant");
    return a[0];
}

// ---------------------------------------------------------------------------
// Signatures
// ---------------------------------------------------------------------------
static size_t type_len(const std::string& s, size_t pos) {
    if (pos >= s.size()) throw std::runtime_error("truncated dbus signature");
    char c = s[pos];
    if (c == 'a') return 1 + type_len(s, pos + 1);
    if (c == '(' || c == '{') {
        char close = c == '(' ? ')' : '}';
        size_t p = pos + 1;
        while (p < s.size() && s[p] != close) p += type_len(s, p);
        if (p >= s.size()) throw std::runtime_error("unbalanced dbus signature");
        return p - pos + 1;
    }
    if (std::strchr("ybnqiuxtdsogvh", c)) return 1;
    throw std::runtime_error(std::string("unsupported dbus type '") + c + "'");
}

static std::vector<std::string> split_sig(const std::string& s) {
    std::vector<std::string> out;
    for (size_t p = 0; p < s.size();) {
        size_t n = type_len(s, p);
        out.push_back(s.substr(p, n));
        p += n;
    }
    return out;
}

static size_t align_of(char c) {
    switch (c) {
        case 'y': case 'g': case 'v': return 1;
        case 'n': case 'q': return 2;
        case 'b': case 'i': case 'u': case 's': case 'o': case 'a': case 'h': return 4;
        default: return 8;  // x t d ( {
    }
}

// ---------------------------------------------------------------------------
// Marshalling (little endian)
// ---------------------------------------------------------------------------
namespace {
struct Writer {
    std::vector<uint8_t>& b;
    void pad(size_t a) {
        while (b.size() % a) b.push_back(0);
    }
    void u8(uint8_t x) { b.push_back(x); }
    void u32(uint32_t x) {
        pad(4);
        for (int i = 0; i < 4; ++i) b.push_back(uint8_t(x >> (8 * i)));
    }
    void u64(uint64_t x) {
        pad(8);
        for (int i = 0; i < 8; ++i) b.push_back(uint8_t(x >> (8 * i)));
    }
    void str(const std::string& s) {
        u32(uint32_t(s.size()));
        b.insert(b.end(), s.begin(), s.end());
        b.push_back(0);
    }
    void sig(const std::string& s) {
        u8(uint8_t(s.size()));
        b.insert(b.end(), s.begin(), s.end());
        b.push_back(0);
    }
    void value(const std::string& t, const Value& v) {
        switch (t[0]) {
            case 'y': u8(std::get<uint8_t>(v.v)); break;
            case 'b': u32(std::get<bool>(v.v) ? 1 : 0); break;
            case 'i': u32(uint32_t(std::get<int32_t>(v.v))); break;
            case 'u': u32(std::get<uint32_t>(v.v)); break;
            case 'x': u64(uint64_t(std::get<int64_t>(v.v))); break;
            case 't': u64(std::get<uint64_t>(v.v)); break;
            case 'd': {
                double d = std::get<double>(v.v);
                uint64_t x;
                std::memcpy(&x, &d, 8);
                u64(x);
                break;
            }
            case 's': case 'o': str(std::get<std::string>(v.v)); break;
            case 'g': sig(std::get<std::string>(v.v)); break;
            case 'v': {
                const Value& inner = v.variant_inner();
                sig(inner.sig);
                value(inner.sig, inner);
                break;
            }
            case 'a': {
                std::string elem = t.substr(1);
                u32(0);
                size_t len_at = b.size() - 4;
                pad(align_of(elem[0]));
                size_t start = b.size();
                for (const auto& e : v.as_array()) value(elem, e);
                uint32_t n = uint32_t(b.size() - start);
                std::memcpy(&b[len_at], &n, 4);
                break;
            }
            case '(': case '{': {
                pad(8);
                auto members = split_sig(t.substr(1, t.size() - 2));
                const auto& a = v.as_array();
                if (a.size() != members.size()) throw std::runtime_error("dbus struct arity mismatch");
                for (size_t i = 0; i < members.size(); ++i) value(members[i], a[i]);
                break;
            }
            default: throw std::runtime_error("cannot marshal dbus type " + t);
        }
    }
};

struct Reader {
    const uint8_t* d;
    size_t n;
    size_t p;
    void need(size_t k) {
        if (p + k > n) throw std::runtime_error("truncated dbus message");
    }
    void pad(size_t a) {
        while (p % a) {
            need(1);
            ++p;
        }
    }
    uint8_t u8() {
        need(1);
        return d[p++];
    }
    uint32_t u32() {
        pad(4);
        need(4);
        uint32_t x;
        std::memcpy(&x, d + p, 4);
        p += 4;
        return x;
    }
    uint64_t u64() {
        pad(8);
        need(8);
        uint64_t x;
        std::memcpy(&x, d + p, 8);
        p += 8;
        return x;
    }
    std::string str() {
        uint32_t len = u32();
        need(size_t(len) + 1);
        std::string s(reinterpret_cast<const char*>(d + p), len);
        p += len + 1;
        return s;
    }
    std::string sig() {
        uint8_t len = u8();
        need(size_t(len) + 1);
        std::string s(reinterpret_cast<const char*>(d + p), len);
        p += size_t(len) + 1;
        return s;
    }
    Value value(const std::string& t, int depth = 0) {
        if (depth > 32) throw std::runtime_error("dbus value nested too deeply");
        Value v;
        v.sig = t;
        switch (t[0]) {
            case 'y': v.v = u8(); break;
            case 'b': v.v = u32() != 0; break;
            case 'n': { pad(2); need(2); int16_t x; std::memcpy(&x, d + p, 2); p += 2; v.v = int32_t(x); break; }
            case 'q': { pad(2); need(2); uint16_t x; std::memcpy(&x, d + p, 2); p += 2; v.v = uint32_t(x); break; }
            case 'i': v.v = int32_t(u32()); break;
            case 'u': case 'h': v.v = u32(); break;
            case 'x': v.v = int64_t(u64()); break;
            case 't': v.v = u64(); break;
            case 'd': {
                uint64_t x = u64();
                double dd;
                std::memcpy(&dd, &x, 8);
                v.v = dd;
                break;
            }
            case 's': case 'o': v.v = str(); break;
            case 'g': v.v = sig(); break;
            case 'v': {
                std::string inner = sig();
                if (split_sig(inner).size() != 1) throw std::runtime_error("bad variant signature");
                v.v = std::make_shared<Array>(Array{value(inner, depth + 1)});
                break;
            }
            case 'a': {
                uint32_t len = u32();
                std::string elem = t.substr(1);
                pad(align_of(elem[0]));
                size_t end = p + len;
                if (end > n) throw std::runtime_error("dbus array overruns message");
                auto arr = std::make_shared<Array>();
                while (p < end) arr->push_back(value(elem, depth + 1));
                v.v = arr;
                break;
            }
            case '(': case '{': {
                pad(8);
                auto arr = std::make_shared<Array>();
                for (auto& m : split_sig(t.substr(1, t.size() - 2))) arr->push_back(value(m, depth + 1));
                v.v = arr;
                break;
            }
            default: throw std::runtime_error("cannot unmarshal dbus type " + t);
        }
        return v;
    }
};
}  // namespace

std::vector<uint8_t> marshal(const Message& m) {
    std::vector<uint8_t> body;
    Writer bw{body};
    auto sigs = split_sig(m.signature);
    if (sigs.size() != m.body.size()) throw std::runtime_error("dbus body does not match signature");
    for (size_t i = 0; i < sigs.size(); ++i) bw.value(sigs[i], m.body[i]);

    std::vector<uint8_t> out;
    Writer w{out};
    w.u8('l');
    w.u8(m.type);
    w.u8(m.flags);
    w.u8(1);
    w.u32(uint32_t(body.size()));
    w.u32(m.serial);
    Array fields;
    auto field = [&](uint8_t code, const Value& v) {
        fields.push_back(Value{"(yv)", std::make_shared<Array>(Array{Value{"y", code}, Value::variant(v)})});
    };
    if (!m.path.empty()) field(1, Value::path(m.path));
    if (!m.interface.empty()) field(2, Value::str(m.interface));
    if (!m.member.empty()) field(3, Value::str(m.member));
    if (!m.error_name.empty()) field(4, Value::str(m.error_name));
    if (m.reply_serial) field(5, Value::u32(m.reply_serial));
    if (!m.destination.empty()) field(6, Value::str(m.destination));
    if (!m.sender.empty()) field(7, Value::str(m.sender));
    if (!m.signature.empty()) field(8, Value{"g", m.signature});
    w.value("a(yv)", Value{"a(yv)", std::make_shared<Array>(fields)});
    w.pad(8);
    out.insert(out.end(), body.begin(), body.end());
    return out;
}

size_t unmarshal(const uint8_t* data, size_t len, Message* out) {
    if (len < 16) return 0;
    if (data[0] != 'l') throw std::runtime_error("big-endian dbus messages are not supported");
    uint32_t body_len, fields_len;
    std::memcpy(&body_len, data + 4, 4);
    std::memcpy(&fields_len, data + 12, 4);
    if (fields_len > (1u << 26) || body_len > (1u << 27)) throw std::runtime_error("dbus message too large");
    size_t hdr_end = 16 + fields_len;
    size_t body_start = (hdr_end + 7) & ~size_t(7);
    size_t total = body_start + body_len;
    if (len < total) return 0;

    Message m;
    m.type = data[1];
    m.flags = data[2];
    std::memcpy(&m.serial, data + 8, 4);
    Reader r{data, hdr_end, 12};
    Value fields = r.value("a(yv)");
    for (const auto& f : fields.as_array()) {
        const auto& st = f.as_array();
        uint8_t code = std::get<uint8_t>(st[0].v);
        const Value& val = st[1].variant_inner();
        switch (code) {
            case 1: m.path = val.as_string(); break;
            case 2: m.interface = val.as_string(); break;
            case 3: m.member = val.as_string(); break;
            case 4: m.error_name = val.as_string(); break;
            case 5: m.reply_serial = val.as_u32(); break;
            case 6: m.destination = val.as_string(); break;
            case 7: m.sender = val.as_string(); break;
            case 8: m.signature = val.as_string(); break;
            default: break;
        }
    }
    Reader br{data + body_start, body_len, 0};
    for (auto& s : split_sig(m.signature)) m.body.push_back(br.value(s));
    *out = std::move(m);
    return total;
}

// ---------------------------------------------------------------------------
// Connection
// ---------------------------------------------------------------------------
std::string Connection::system_bus_address() {
    const char* a = std::getenv("DBUS_SYSTEM_BUS_ADDRESS");
    return (a && *a) ? a : "unix:path=/var/run/dbus/system_bus_socket";
}

Connection::Connection(const std::string& address, int timeout_ms) : timeout_ms_(timeout_ms) {
    std::string path = address;
    if (path.rfind("unix:", 0) == 0) {
        path.clear();
        for (auto& kv : split(address.substr(5), ',')) {
            if (kv.rfind("path=", 0) == 0) path = kv.substr(5);
        }
        if (path.empty()) throw std::runtime_error("unsupported D-Bus address " + address);
    }
    fd_ = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd_ < 0) throw_errno("socket(AF_UNIX)");
    sockaddr_un sa{};
    sa.sun_family = AF_UNIX;
    if (path.size() >= sizeof sa.sun_path) throw std::runtime_error("D-Bus socket path too long");
    std::memcpy(sa.sun_path, path.c_str(), path.size());
    if (::connect(fd_, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
        int e = errno;
        ::close(fd_);
        fd_ = -1;
        throw SysError(e, "connect " + path);
    }
    // SASL EXTERNAL with our uid, hex-encoded ASCII decimal.
    std::string uid = std::to_string(::getuid()), hex;
    for (char c : uid) hex += strfmt("%02x", static_cast<unsigned char>(c));
    if (::write(fd_, "\0", 1) != 1) throw_errno("dbus auth nul");
    send_line("AUTH EXTERNAL " + hex + "\r\n");
    std::string resp = read_line();
    if (resp.rfind("OK", 0) != 0) throw DBusError("org.freedesktop.DBus.Error.AuthFailed", resp);
    send_line("BEGIN\r\n");
    auto r = call("org.freedesktop.DBus", "/org/freedesktop/DBus", "org.freedesktop.DBus", "Hello");
    if (!r.empty()) unique_name_ = r[0].as_string();
}

Connection::~Connection() {
    if (fd_ >= 0) ::close(fd_);
}

void Connection::send_line(const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
        ssize_t n = ::write(fd_, s.data() + off, s.size() - off);
        if (n < 0) {
            if (errno == EINTR) continue;
            throw_errno("dbus write");
        }
        off += size_t(n);
    }
}

static void wait_readable(int fd, int timeout_ms) {
    pollfd p{fd, POLLIN, 0};
    int r;
    do {
        r = ::poll(&p, 1, timeout_ms);
    } while (r < 0 && errno == EINTR);
    if (r < 0) throw_errno("dbus poll");
    if (r == 0) throw DBusError("org.freedesktop.DBus.Error.Timeout", "no reply");
}

std::string Connection::read_line() {
    std::string line;
    for (;;) {
        auto it = std::find(rbuf_.begin(), rbuf_.end(), '\n');
        if (it != rbuf_.end()) {
            line.assign(rbuf_.begin(), it);
            rbuf_.erase(rbuf_.begin(), it + 1);
            if (!line.empty() && line.back() == '\r') line.pop_back();
            return line;
        }
        wait_readable(fd_, timeout_ms_);
        uint8_t buf[512];
        ssize_t n = ::read(fd_, buf, sizeof buf);
        if (n <= 0) throw std::runtime_error("dbus connection closed during auth");
        rbuf_.insert(rbuf_.end(), buf, buf + n);
    }
}

Message Connection::read_message() {
    for (;;) {
        if (!rbuf_.empty()) {
            Message m;
            size_t used = unmarshal(rbuf_.data(), rbuf_.size(), &m);
            if (used) {
                rbuf_.erase(rbuf_.begin(), rbuf_.begin() + long(used));
                return m;
            }
        }
        wait_readable(fd_, timeout_ms_);
        uint8_t buf[8192];
        ssize_t n = ::read(fd_, buf, sizeof buf);
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) throw std::runtime_error("dbus connection closed");
        rbuf_.insert(rbuf_.end(), buf, buf + n);
    }
}

std::vector<Value> Connection::call(const std::string& dest, const std::string& path, const std::string& iface,
                                    const std::string& member, const std::string& signature,
                                    const std::vector<Value>& args) {
    Message m;
    m.type = 1;
    m.serial = serial_++;
    m.destination = dest;
    m.path = path;
    m.interface = iface;
    m.member = member;
    m.signature = signature;
    m.body = args;
    auto bytes = marshal(m);
    send_line(std::string(bytes.begin(), bytes.end()));
    for (;;) {
        Message r = read_message();
        if (r.reply_serial != m.serial) continue;  // signals / unrelated
        if (r.type == 3) {
            std::string msg = !r.body.empty() && r.body[0].sig == "s" ? r.body[0].as_string() : "";
            throw DBusError(r.error_name, msg);
        }
        return r.body;
    }
}

Value Connection::get_property(const std::string& dest, const std::string& path, const std::string& iface,
                               const std::string& prop) {
    auto r = call(dest, path, "org.freedesktop.DBus.Properties", "Get", "ss", {Value::str(iface), Value::str(prop)});
    if (r.empty()) throw std::runtime_error("empty Properties.Get reply");
    return r[0].variant_inner();
}

void Connection::set_property(const std::string& dest, const std::string& path, const std::string& iface,
                              const std::string& prop, const Value& v) {
    call(dest, path, "org.freedesktop.DBus.Properties", "Set", "ssv",
         {Value::str(iface), Value::str(prop), Value::variant(v)});
}

}  // namespace netop::dbus
