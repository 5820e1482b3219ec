// ethtool private flags (SIOCETHTOOL) — turning off a NIC firmware's own LLDP agent.
//
// Several RoCE NIC families run an LLDP/DCBX agent in firmware that consumes the switch's
// LLDPDUs before the host sees them; an AF_PACKET listener then waits for nothing
// (SURVEY.md §7.7 "hard part 1").  The reference has no answer to this (pkg/lldp/client.go
// just times out after --wait).  The agent's `--disable-fw-lldp` looks up the driver's
// private flags and flips the known "firmware LLDP" flag for the duration of its run,
// restoring the original value on exit:
//
//   i40e (X710/XL710):      disable-fw-lldp = on
//   ice  (E810):            fw-lldp-agent   = off
//   anything else:          --fw-lldp-priv-flag NAME=0|1 (site-specific)
//
// mlx5 (ConnectX) and ionic (Pensando): no private flag is known to the agent; a firmware
// LLDP agent there is a persistent NIC setting outside the scope of a DaemonSet (unverified on
// this pool: parity unpinned).  The agent reports "no firmware LLDP flag" for them, and a NIC
// that stays silent is diagnosed after --wait (Agent::diagnose_silent).
#pragma once

#include <cstdint>
#include <memory>
#include <optional>
#include <string>
#include <vector>

namespace netop::ethtool {

struct PrivFlags {
    std::vector<std::string> names;  // bit i <-> names[i]
    uint32_t bits = 0;
    int index_of(const std::string& name) const;
};

// Injectable operation table (real ioctl implementation, fakes in tests).
class Ops {
   public:
    virtual ~Ops() = default;
    virtual std::string driver(const std::string& ifname) = 0;     // "" when unknown
    virtual PrivFlags get(const std::string& ifname) = 0;           // throws SysError
    virtual void set(const std::string& ifname, uint32_t bits) = 0;  // throws SysError
};

std::unique_ptr<Ops> make_ioctl_ops();

struct FlagRule {
    std::string name;
    bool value = true;  // desired state while the agent runs
};

// Built-in rules (above) plus user rules "NAME=0|1[,NAME=0|1...]"; throws on bad syntax.
std::vector<FlagRule> parse_rules(const std::string& spec);
std::vector<FlagRule> builtin_rules();

struct FwLldpResult {
    std::string ifname;
    std::string driver;
    std::string flag;          // flag that was changed ("" = none applicable)
    bool changed = false;
    uint32_t original_bits = 0;
    std::string error;         // non-empty on failure
    std::string summary() const;
};

// Applies the first matching rule on `ifname`; never throws (errors land in .error).
FwLldpResult disable_fw_lldp(Ops& ops, const std::string& ifname, const std::vector<FlagRule>& rules);
// Puts back the original private flags if disable_fw_lldp changed them.
void restore(Ops& ops, const FwLldpResult& r);

}  // namespace netop::ethtool
