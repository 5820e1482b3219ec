// ethtool private flags (SIOCETHTOOL) — turning off a NIC firmware's own LLDP agent.
//
// Several RoCE NIC families run an LLDP/DCBX agent in firmware that consumes the switch's
// LLDPDUs before the host sees them; an AF_PACKET listener then waits for nothing
// (SURVEY.md §7.7 "hard part 1").  The reference has no answer to this (pkg/lldp/client.go
// just times out after --wait).  The agent's `--disable-fw-lldp` looks up the driver's
// private flags and flips the known "firmware LLDP" flag for the duration of its run,
// restoring the original value when it exits cleanly (an agent that fails leaves them, like its
// addresses, to the agent the kubelet restarts, so a crash loop does not flip them every time;
// the originals wait in --fw-lldp-state meanwhile, and under --keep-config until --cleanup):
//
//   i40e (X710/XL710):      disable-fw-lldp = on
//   ice  (E810):            fw-lldp-agent   = off
//   anything else:          --fw-lldp-priv-flag NAME=0|1 (site-specific)
//
// mlx5 (ConnectX) and ionic (Pensando): no private flag is known to the agent.  For a NIC
// without one, the driver-neutral signal is its DCBX mode (DCB netlink, DCB_CMD_GDCBX): without
// DCB_CAP_DCBX_HOST, an embedded agent runs DCBX, and with it the port's LLDP exchange.  Per
// the drivers' dcbnl code, ice and i40e report DCB_CAP_DCBX_LLD_MANAGED while their firmware
// agent runs, and mlx5_core reports no HOST bit in its firmware ("auto") DCBX mode and moves to
// host mode on DCB_CMD_SDCBX with HOST set.  Handing DCBX to the host on such a NIC is a separate
// opt-in (`--fw-lldp-dcbx-host`, policy `handDcbxToHost`): the firmware then stops negotiating
// PFC/ETS with the switch, which lossless RoCE depends on unless the host runs a DCBX agent of its
// own, and whether it makes mlx5 firmware pass LLDPDUs up is unverified on this pool (parity
// unpinned; the box's NICs live outside its network namespace).  Without it `--disable-fw-lldp`
// only reads the DCBX mode there.  The original mode goes back on exit.  A NIC that stays silent
// is diagnosed after --wait with its DCBX mode (Agent::diagnose_silent).
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
    // DCBX mode (DCB_CAP_DCBX_* bits); nullopt when the NIC has no DCB interface.
    virtual std::optional<uint8_t> dcbx_get(const std::string& ifname) {
        (void)ifname;
        return std::nullopt;
    }
    // false when the driver refused the mode; throws SysError.
    virtual bool dcbx_set(const std::string& ifname, uint8_t mode);
};

// DCBX mode bits in words: "0x0c (firmware, cee, ieee)", "0x09 (host, ieee)".
std::string dcbx_str(uint8_t mode);
// An embedded (NIC-firmware or LLD) agent runs DCBX and the port's LLDP: no DCB_CAP_DCBX_HOST.
bool dcbx_embedded(uint8_t mode);

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
    std::optional<uint8_t> dcbx;  // DCBX mode found (nullopt: no DCB interface, or not asked)
    bool dcbx_changed = false;    // the agent handed DCBX to the host
    bool dry_run = false;         // inspected only (--dry-run): nothing was set
    bool would_change = false;    // dry run: the flag / DCBX mode would be changed
    std::string error;         // non-empty on failure
    std::string summary() const;
};

// Applies the first matching rule on `ifname`; with no applicable private flag, reads the DCBX
// mode and, only with hand_dcbx, hands an embedded DCBX agent's port to the host
// (DCB_CMD_SDCBX).  Never throws (errors land in .error).  With apply = false (the agent's
// --dry-run) nothing is set: .would_change says what would be.
FwLldpResult disable_fw_lldp(Ops& ops, const std::string& ifname, const std::vector<FlagRule>& rules,
                             bool apply = true, bool hand_dcbx = false);
// Puts back the original private flags / DCBX mode if disable_fw_lldp changed them; false when
// any of it could not be put back (e.g. the interface is gone or was renamed).
bool restore(Ops& ops, const FwLldpResult& r);

// The originals of what was changed, kept on the node across agent restarts (--keep-config
// with --fw-lldp-state): one line per change, "<ifname> priv 0x<bits>" or "<ifname> dcbx
// 0x<mode>".  decode_state skips lines it does not understand.
std::string encode_state(const std::vector<FwLldpResult>& rs);
std::vector<FwLldpResult> decode_state(const std::string& text);

}  // namespace netop::ethtool
