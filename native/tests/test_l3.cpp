#include "check.hpp"
#include "netop/l3.hpp"

using namespace netop;
using namespace netop::l3;

TEST(l3_reference_token1) {
    std::string err;
    auto a = parse_port_description("no-alert 10.200.10.2/30", TokenPolicy::Compat, &err);
    CHECK(a);
    CHECK_EQ(a->peer.str(), std::string("10.200.10.2"));
    CHECK_EQ(a->local.str(), std::string("10.200.10.1"));
    CHECK_EQ(a->p2p_network().str(), std::string("10.200.10.0/30"));
    CHECK_EQ(a->routed_network().str(), std::string("10.200.0.0/16"));
    // peer .1 -> local .2
    a = parse_port_description("x 10.0.0.1/30", TokenPolicy::Compat, &err);
    CHECK_EQ(a->local.str(), std::string("10.0.0.2"));
}

TEST(l3_reference_errors) {
    std::string err;
    CHECK(!parse_port_description("no-address", TokenPolicy::Compat, &err));
    CHECK(err.find("could not split") != std::string::npos);
    CHECK(!parse_port_description("a garbage", TokenPolicy::Compat, &err));
    CHECK(!parse_port_description("a 10.0.0.2/24", TokenPolicy::Compat, &err));
    CHECK(err.find("mask is 24") != std::string::npos);
    // Go strings.Split on a single space: a double space makes token [1] empty.
    CHECK(!parse_port_description("a  10.0.0.2/30", TokenPolicy::Compat, &err));
    // Network / broadcast address of the /30 are rejected.
    CHECK(!parse_port_description("a 10.0.0.0/30", TokenPolicy::Compat, &err));
    CHECK(!parse_port_description("a 10.0.0.3/30", TokenPolicy::Compat, &err));
}

TEST(l3_last_token_fallback) {
    std::string err;
    // README says the address is "at the end": accept it when token [1] is not an address.
    auto a = parse_port_description("to leaf1 eth1/1 10.1.1.2/30", TokenPolicy::CompatThenLast, &err);
    CHECK(a);
    CHECK_EQ(a->local.str(), std::string("10.1.1.1"));
    a = parse_port_description("a  10.0.0.2/30", TokenPolicy::CompatThenLast, &err);
    CHECK(a);
    CHECK(!parse_port_description("to leaf1 eth1/1 10.1.1.2/30", TokenPolicy::Compat, &err));
    CHECK(!parse_port_description("", TokenPolicy::CompatThenLast, &err));
    // token [1] wins when valid even if the last token is also an address.
    a = parse_port_description("x 10.0.0.2/30 10.9.9.2/30", TokenPolicy::CompatThenLast, &err);
    CHECK_EQ(a->peer.str(), std::string("10.0.0.2"));
}

TEST(l3_any_token) {
    std::string err;
    auto a = parse_port_description("uplink=10.5.5.6/30 via tor", TokenPolicy::AnyToken, &err);
    CHECK(!a);  // "uplink=10.5.5.6/30" is not a bare CIDR
    a = parse_port_description("uplink 7 10.5.5.6/30 via tor", TokenPolicy::AnyToken, &err);
    CHECK(a);
    CHECK_EQ(a->local.str(), std::string("10.5.5.5"));
    CHECK_EQ(mask_string(30), std::string("255.255.255.252"));
}

TEST(l3_exhaustive_last_octet) {
    std::string err;
    for (int o = 0; o < 256; ++o) {
        auto a = parse_port_description("t 172.16.3." + std::to_string(o) + "/30", TokenPolicy::Compat, &err);
        int host = o & 3;
        if (host == 1 || host == 2) {
            CHECK(a);
            CHECK_EQ(int(a->local.v & 0xff), o ^ 3);
            CHECK(a->p2p_network().contains(a->local));
            CHECK(a->p2p_network().contains(a->peer));
        } else {
            CHECK(!a);
        }
    }
}
