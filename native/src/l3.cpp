#include "netop/l3.hpp"

namespace netop::l3 {

static std::optional<P2pAddressing> from_cidr(std::string_view token, std::string* err) {
    auto pfx = Ipv4Prefix::parse(token);
    if (!pfx) {
        if (err) *err = "could not parse '" + std::string(token) + "' as an IPv4 CIDR";
        return std::nullopt;
    }
    if (pfx->len != kPointToPointMask) {
        if (err) *err = strfmt("mask is %d, not the expected %d", pfx->len, kPointToPointMask);
        return std::nullopt;
    }
    uint32_t host = pfx->addr.v & 0x3u;
    if (host == 0 || host == 3) {
        if (err) *err = "peer " + pfx->addr.str() + " is the /30 network or broadcast address";
        return std::nullopt;
    }
    P2pAddressing a;
    a.peer = pfx->addr;
    a.local = Ipv4{pfx->addr.v ^ 0x3u};
    a.prefix = kPointToPointMask;
    return a;
}

std::optional<P2pAddressing> parse_port_description(std::string_view desc, TokenPolicy policy, std::string* err) {
    std::string e1;
    if (policy == TokenPolicy::AnyToken) {
        for (const auto& t : split_ws(desc)) {
            if (t.find('/') == std::string::npos) continue;
            auto a = from_cidr(t, &e1);
            if (a) return a;
        }
        if (err) *err = e1.empty() ? "no CIDR token in port description '" + std::string(desc) + "'" : e1;
        return std::nullopt;
    }

    auto parts = split(desc, ' ');
    std::optional<P2pAddressing> first;
    if (parts.size() >= 2) {
        first = from_cidr(parts[1], &e1);
        if (first || policy == TokenPolicy::Compat) {
            if (!first && err) *err = e1;
            return first;
        }
    } else if (policy == TokenPolicy::Compat) {
        if (err) *err = "could not split string '" + std::string(desc) + "'";
        return std::nullopt;
    }
    auto fields = split_ws(desc);
    if (fields.empty()) {
        if (err) *err = "empty port description";
        return std::nullopt;
    }
    std::string e2;
    auto last = from_cidr(fields.back(), &e2);
    if (!last && err) *err = e1.empty() ? e2 : e1 + "; last token: " + e2;
    return last;
}

std::string mask_string(int prefix) { return Ipv4{prefix_mask(prefix)}.str(); }

std::optional<TokenPolicy> parse_token_policy(std::string_view s) {
    if (s == "compat" || s == "index1") return TokenPolicy::Compat;
    if (s == "compat-then-last" || s == "default" || s.empty()) return TokenPolicy::CompatThenLast;
    if (s == "any") return TokenPolicy::AnyToken;
    return std::nullopt;
}

}  // namespace netop::l3
