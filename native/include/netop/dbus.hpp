// Minimal D-Bus wire-protocol client (no libdbus): SASL EXTERNAL auth, Hello,
// method calls with the handful of types NetworkManager needs (s, o, g, b, u, i, v, a*),
// and reply / error matching by serial.
//
// The reference reaches NetworkManager through godbus + gonetworkmanager
// (reference internal/nm/networkmanager.go:22,44-77).  libdbus headers are not present
// in this image and the node agent must stay dependency-free, so the protocol subset
// is implemented directly (D-Bus Specification, "Message Protocol").
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <variant>
#include <vector>

namespace netop::dbus {

struct Value;
using Array = std::vector<Value>;

// A demarshalled D-Bus value.  `sig` is the single complete type of the value.
struct Value {
    std::string sig;
    std::variant<std::monostate, bool, uint8_t, int32_t, uint32_t, int64_t, uint64_t, double, std::string,
                 std::shared_ptr<Array>>
        v;

    static Value str(const std::string& s) { return Value{"s", s}; }
    static Value path(const std::string& s) { return Value{"o", s}; }
    static Value boolean(bool b) { return Value{"b", b}; }
    static Value u32(uint32_t x) { return Value{"u", x}; }
    static Value variant(const Value& inner) { return Value{"v", std::make_shared<Array>(Array{inner})}; }

    const std::string& as_string() const;
    bool as_bool() const;
    uint32_t as_u32() const;
    const Array& as_array() const;     // arrays, structs
    const Value& variant_inner() const;
};

struct Message {
    uint8_t type = 1;  // 1 call, 2 return, 3 error, 4 signal
    uint8_t flags = 0;
    uint32_t serial = 0;
    uint32_t reply_serial = 0;
    std::string path, interface, member, error_name, destination, sender, signature;
    std::vector<Value> body;
};

std::vector<uint8_t> marshal(const Message& m);
// Parses one complete message from `data`; returns bytes consumed or 0 if incomplete.
size_t unmarshal(const uint8_t* data, size_t len, Message* out);

class DBusError : public std::runtime_error {
   public:
    DBusError(const std::string& name, const std::string& msg) : std::runtime_error(name + ": " + msg), name_(name) {}
    const std::string& name() const { return name_; }

   private:
    std::string name_;
};

class Connection {
   public:
    // address: "unix:path=/var/run/dbus/system_bus_socket" (also accepts a bare path).
    explicit Connection(const std::string& address, int timeout_ms = 5000);
    ~Connection();
    static std::string system_bus_address();  // $DBUS_SYSTEM_BUS_ADDRESS or the default socket

    std::vector<Value> call(const std::string& dest, const std::string& path, const std::string& iface,
                            const std::string& member, const std::string& signature = "",
                            const std::vector<Value>& args = {});
    const std::string& unique_name() const { return unique_name_; }

    // org.freedesktop.DBus.Properties helpers
    Value get_property(const std::string& dest, const std::string& path, const std::string& iface,
                       const std::string& prop);
    void set_property(const std::string& dest, const std::string& path, const std::string& iface,
                      const std::string& prop, const Value& v);

   private:
    void send_line(const std::string& s);
    std::string read_line();
    Message read_message();

    int fd_ = -1;
    int timeout_ms_;
    uint32_t serial_ = 1;
    std::string unique_name_;
    std::vector<uint8_t> rbuf_;
};

}  // namespace netop::dbus
