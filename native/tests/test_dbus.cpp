#include "check.hpp"
#include "netop/dbus.hpp"

using namespace netop::dbus;

TEST(dbus_marshal_roundtrip) {
    Message m;
    m.type = 1;
    m.serial = 42;
    m.destination = "org.freedesktop.NetworkManager";
    m.path = "/org/freedesktop/NetworkManager/Devices/3";
    m.interface = "org.freedesktop.DBus.Properties";
    m.member = "Set";
    m.signature = "ssv";
    m.body = {Value::str("org.freedesktop.NetworkManager.Device"), Value::str("Managed"), Value::variant(Value::boolean(false))};
    auto b = marshal(m);
    CHECK_EQ(b.size() % 1, size_t(0));
    Message r;
    size_t used = unmarshal(b.data(), b.size(), &r);
    CHECK_EQ(used, b.size());
    CHECK_EQ(r.serial, uint32_t(42));
    CHECK_EQ(r.member, std::string("Set"));
    CHECK_EQ(r.path, m.path);
    CHECK_EQ(r.signature, std::string("ssv"));
    CHECK_EQ(r.body.size(), size_t(3));
    CHECK_EQ(r.body[1].as_string(), std::string("Managed"));
    CHECK_EQ(r.body[2].variant_inner().as_bool(), false);
    // Incomplete buffers report 0 consumed.
    CHECK_EQ(unmarshal(b.data(), b.size() - 1, &r), size_t(0));
}

TEST(dbus_arrays_and_structs) {
    Message m;
    m.type = 2;
    m.serial = 7;
    m.reply_serial = 3;
    m.signature = "aoa{sv}(ut)";
    auto paths = std::make_shared<Array>(Array{Value::path("/a/1"), Value::path("/a/22"), Value::path("/a/333")});
    auto dict = std::make_shared<Array>(Array{
        Value{"{sv}", std::make_shared<Array>(Array{Value::str("Version"), Value::variant(Value::str("1.46"))})},
        Value{"{sv}", std::make_shared<Array>(Array{Value::str("State"), Value::variant(Value::u32(70))})}});
    auto st = std::make_shared<Array>(Array{Value::u32(5), Value{"t", uint64_t(1) << 40}});
    m.body = {Value{"ao", paths}, Value{"a{sv}", dict}, Value{"(ut)", st}};
    auto b = marshal(m);
    Message r;
    CHECK_EQ(unmarshal(b.data(), b.size(), &r), b.size());
    CHECK_EQ(r.reply_serial, uint32_t(3));
    CHECK_EQ(r.body[0].as_array().size(), size_t(3));
    CHECK_EQ(r.body[0].as_array()[2].as_string(), std::string("/a/333"));
    CHECK_EQ(r.body[1].as_array()[1].as_array()[1].variant_inner().as_u32(), uint32_t(70));
    CHECK_EQ(std::get<uint64_t>(r.body[2].as_array()[1].v), uint64_t(1) << 40);
    // Empty array of 8-aligned elements.
    m.signature = "a(ut)";
    m.body = {Value{"a(ut)", std::make_shared<Array>()}};
    b = marshal(m);
    CHECK_EQ(unmarshal(b.data(), b.size(), &r), b.size());
    CHECK(r.body[0].as_array().empty());
}

TEST(dbus_rejects_garbage) {
    std::vector<uint8_t> junk(64, 0xff);
    junk[0] = 'l';
    Message r;
    CHECK_THROWS(unmarshal(junk.data(), junk.size(), &r));
    junk[0] = 'B';
    CHECK_THROWS(unmarshal(junk.data(), junk.size(), &r));
}
