// L3 point-to-point addressing derived from the switch's LLDP Port Description.
//
// Reference behaviour (cmd/discover/network.go:141-173): split the Port Description
// on " " and parse token [1] as a CIDR; require /30; local = peer XOR 0x3.
// README.md:23 of the reference says the address is "at the end" of the string, so
// in addition to the reference's token [1] we accept the last whitespace-separated
// token (TokenPolicy::CompatThenLast, the default).  A peer that is the /30 network
// or broadcast address is rejected (the reference would configure the broadcast /
// network address as the local IP).
#pragma once

#include <optional>
#include <string>
#include <string_view>

#include "netop/common.hpp"

namespace netop::l3 {

constexpr int kPointToPointMask = 30;  // RouteMaskPointToPoint (network.go:315)
constexpr int kRoutedNetworkMask = 16; // RouteMaskRoutedNetwork (network.go:314)

enum class TokenPolicy {
    Compat,          // token [1] of strings.Split(desc, " ") only (exact reference behaviour)
    CompatThenLast,  // token [1], falling back to the last whitespace-separated token
    AnyToken,        // the first token that parses as an IPv4 CIDR
};

struct P2pAddressing {
    Ipv4 peer;   // switch-side address (gateway)
    Ipv4 local;  // our address = peer ^ 3
    int prefix = kPointToPointMask;

    Ipv4Prefix local_prefix() const { return Ipv4Prefix{local, prefix}; }
    Ipv4Prefix p2p_network() const { return Ipv4Prefix{local, prefix}.masked(); }
    Ipv4Prefix routed_network() const { return Ipv4Prefix{local, kRoutedNetworkMask}.masked(); }
};

// Returns nullopt and fills `err` with a human-readable reason on failure.
std::optional<P2pAddressing> parse_port_description(std::string_view desc, TokenPolicy policy, std::string* err);

// Subnet mask string for the /30 ("255.255.255.252"), as written to the RCCL artifact.
std::string mask_string(int prefix);

std::optional<TokenPolicy> parse_token_policy(std::string_view s);

}  // namespace netop::l3
