#include "check.hpp"
#include "netop/lldp.hpp"

using namespace netop;
using namespace netop::lldp;

static std::vector<uint8_t> hex(const char* s) {
    std::vector<uint8_t> out;
    auto v = [](char c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; };
    while (*s) {
        if (*s == ' ') {
            ++s;
            continue;
        }
        out.push_back(uint8_t(v(s[0]) << 4 | v(s[1])));
        s += 2;
    }
    return out;
}

TEST(lldp_roundtrip_switch_frame) {
    auto mac = *MacAddr::parse("02:11:22:33:44:55");
    auto f = make_switch_frame(mac, "tor1", "Ethernet1/1", "no-alert 10.200.10.2/30");
    auto bytes = encode(f);
    CHECK(bytes.size() >= 60);
    DecodeError e;
    auto d = decode(bytes.data(), bytes.size(), &e);
    CHECK(d);
    CHECK_EQ(int(e), int(DecodeError::None));
    CHECK_EQ(*d->port_description, std::string("no-alert 10.200.10.2/30"));
    CHECK_EQ(*d->system_name, std::string("tor1"));
    CHECK_EQ(d->port_id_str(), std::string("Ethernet1/1"));
    CHECK_EQ(d->peer_mac()->str(), std::string("02:11:22:33:44:55"));
    CHECK_EQ(d->ttl, 120);
    CHECK(d->dst == kNearestBridge);
    CHECK(d->src == mac);
}

TEST(lldp_port_mac_overrides_chassis_mac) {
    Frame f;
    f.src = *MacAddr::parse("02:00:00:00:00:01");
    f.chassis_subtype = kChassisMac;
    f.chassis_id = std::string("\x02\x00\x00\x00\x00\x01", 6);
    f.port_subtype = kPortMac;
    f.port_id = std::string("\x02\x00\x00\x00\x00\x02", 6);
    auto d = decode(encode(f).data(), encode(f).size());
    CHECK(d);
    CHECK_EQ(d->peer_mac()->str(), std::string("02:00:00:00:00:02"));
    // Non-MAC subtypes leave the peer MAC unset.
    f.chassis_subtype = kChassisLocal;
    f.port_subtype = kPortIfName;
    auto bytes = encode(f);
    auto d2 = decode(bytes.data(), bytes.size());
    CHECK(d2 && !d2->peer_mac());
}

TEST(lldp_golden_bytes) {
    // Hand-assembled LLDPDU: chassis MAC, port ifName "Eth1/3", TTL 120, port description,
    // system name "leaf1", management address 10.0.0.1, org TLV (IEEE 802.1 port VLAN), end.
    auto b = hex(
        "0180c200000e 020000aabbcc 88cc"
        "0207 04 020000aabbcc"
        "0407 05 457468312f33"
        "0602 0078"
        "0817 6e6f2d616c65727420 31302e3230302e31302e322f3330"  // "no-alert 10.200.10.2/30"
        "0a05 6c65616631"
        "100c 05 01 0a000001 02 00000001 00"
        "fe06 0080c2 01 0064"
        "0000");
    DecodeError e;
    auto d = decode(b.data(), b.size(), &e);
    CHECK(d);
    CHECK_EQ(*d->port_description, std::string("no-alert 10.200.10.2/30"));
    CHECK_EQ(*d->system_name, std::string("leaf1"));
    CHECK_EQ(d->port_id_str(), std::string("Eth1/3"));
    CHECK_EQ(d->management.size(), size_t(1));
    CHECK_EQ(d->management[0].address, std::string("\x0a\x00\x00\x01", 4));
    CHECK_EQ(d->org.size(), size_t(1));
    CHECK_EQ(d->org[0].oui, uint32_t(0x0080c2));
    CHECK_EQ(d->peer_mac()->str(), std::string("02:00:00:aa:bb:cc"));
    // Re-encoding what we decoded yields an equivalent frame.
    auto again = decode(encode(*d).data(), encode(*d).size());
    CHECK(again && *again->port_description == *d->port_description && again->management.size() == 1);
}

TEST(lldp_vlan_tagged) {
    Frame f = make_switch_frame(*MacAddr::parse("02:00:00:00:00:09"), "s", "p", "x 10.0.0.2/30");
    f.vlan = 100;
    auto b = encode(f);
    auto d = decode(b.data(), b.size());
    CHECK(d);
    CHECK_EQ(*d->vlan, uint16_t(100));
    CHECK_EQ(*d->port_description, std::string("x 10.0.0.2/30"));
}

TEST(lldp_rejects_malformed) {
    DecodeError e;
    auto good = encode(make_switch_frame(*MacAddr::parse("02:00:00:00:00:09"), "s", "p", "d"));
    CHECK(!decode(good.data(), 10, &e));
    CHECK_EQ(int(e), int(DecodeError::TooShort));
    auto notlldp = good;
    notlldp[12] = 0x08;
    notlldp[13] = 0x00;
    CHECK(!decode(notlldp.data(), notlldp.size(), &e));
    CHECK_EQ(int(e), int(DecodeError::NotLldp));
    // Missing chassis: first TLV is a port ID.
    auto b = hex("0180c200000e 020000aabbcc 88cc 0407 05 457468312f33 0602 0078 0000");
    CHECK(!decode(b.data(), b.size(), &e));
    CHECK_EQ(int(e), int(DecodeError::MissingChassisId));
    // Missing TTL.
    b = hex("0180c200000e 020000aabbcc 88cc 0207 04 020000aabbcc 0407 05 457468312f33 0000");
    CHECK(!decode(b.data(), b.size(), &e));
    CHECK_EQ(int(e), int(DecodeError::MissingTtl));
    // TLV length overruns the frame.
    b = hex("0180c200000e 020000aabbcc 88cc 02ff 04 020000aabbcc");
    CHECK(!decode(b.data(), b.size(), &e));
    CHECK_EQ(int(e), int(DecodeError::TlvOverrun));
    // Empty chassis ID.
    b = hex("0180c200000e 020000aabbcc 88cc 0201 04 0407 05 457468312f33 0602 0078 0000");
    CHECK(!decode(b.data(), b.size(), &e));
    CHECK_EQ(int(e), int(DecodeError::BadChassisId));
}

TEST(lldp_fuzz_truncations_never_crash) {
    auto f = make_switch_frame(*MacAddr::parse("02:00:00:00:00:09"), "sys", "port", "no-alert 10.1.2.2/30");
    f.management.push_back(ManagementAddress{1, std::string("\x0a\x01\x02\x02", 4), 2, 7, ""});
    f.org.push_back(OrgTlv{0x0080c2, 1, std::string("\x00\x64", 2)});
    auto b = encode(f);
    for (size_t n = 0; n <= b.size(); ++n) (void)decode(b.data(), n);
    // Flip every byte of the TLV area.
    for (size_t i = 14; i < b.size(); ++i) {
        auto c = b;
        c[i] ^= 0xff;
        (void)decode(c.data(), c.size());
    }
}
