// IEEE 802.1AB (LLDP) frame codec.
//
// The reference decodes frames with gopacket's layers.LinkLayerDiscovery(+Info)
// (reference pkg/lldp/client.go:113-140) and extracts: ChassisID (MAC subtype),
// PortID (MAC subtype, overrides the chassis MAC), SysName, SysDescription and
// PortDescription.  This codec decodes the same fields directly from the wire
// bytes (zero-copy views into the receive buffer are converted once), validates
// the mandatory TLV order, and also ENCODES frames: the encoder drives the
// synthetic-switch transmitter used by the netns harness and the fuzz tests.
#pragma once

#include <cstddef>
#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "netop/common.hpp"

namespace netop::lldp {

constexpr uint16_t kEtherType = 0x88cc;
// Nearest-bridge group address; what a switch port sends LLDPDUs to.
extern const MacAddr kNearestBridge;         // 01:80:c2:00:00:0e
extern const MacAddr kNearestNonTpmrBridge;  // 01:80:c2:00:00:03
extern const MacAddr kNearestCustomerBridge; // 01:80:c2:00:00:00

enum TlvType : uint8_t {
    kEnd = 0,
    kChassisId = 1,
    kPortId = 2,
    kTtl = 3,
    kPortDescription = 4,
    kSystemName = 5,
    kSystemDescription = 6,
    kSystemCapabilities = 7,
    kManagementAddress = 8,
    kOrgSpecific = 127,
};

enum ChassisSubtype : uint8_t {
    kChassisComponent = 1,
    kChassisIfAlias = 2,
    kChassisPortComponent = 3,
    kChassisMac = 4,
    kChassisNetworkAddress = 5,
    kChassisIfName = 6,
    kChassisLocal = 7,
};

enum PortSubtype : uint8_t {
    kPortIfAlias = 1,
    kPortComponent = 2,
    kPortMac = 3,
    kPortNetworkAddress = 4,
    kPortIfName = 5,
    kPortAgentCircuitId = 6,
    kPortLocal = 7,
};

struct ManagementAddress {
    uint8_t addr_subtype = 1;  // IANA address family: 1 = IPv4, 2 = IPv6
    std::string address;       // raw bytes
    uint8_t if_subtype = 2;    // 2 = ifIndex
    uint32_t if_number = 0;
    std::string oid;
};

struct OrgTlv {
    uint32_t oui = 0;  // 24-bit
    uint8_t subtype = 0;
    std::string info;
};

struct Frame {
    MacAddr dst = kNearestBridge;
    MacAddr src;
    std::optional<uint16_t> vlan;  // 802.1Q VID when the frame carried a tag

    uint8_t chassis_subtype = kChassisMac;
    std::string chassis_id;  // raw bytes (6 bytes for the MAC subtype)
    uint8_t port_subtype = kPortIfName;
    std::string port_id;     // raw bytes
    uint16_t ttl = 120;

    std::optional<std::string> port_description;
    std::optional<std::string> system_name;
    std::optional<std::string> system_description;
    std::optional<std::pair<uint16_t, uint16_t>> capabilities;  // (system, enabled)
    std::vector<ManagementAddress> management;
    std::vector<OrgTlv> org;

    // Peer MAC the way the reference derives it: ChassisID with the MAC subtype,
    // overridden by a PortID with the MAC subtype (pkg/lldp/client.go:122-128).
    std::optional<MacAddr> peer_mac() const;
    std::string chassis_id_str() const;  // MAC → "aa:bb:..", textual subtypes verbatim
    std::string port_id_str() const;
    // IEEE 802.3 organizationally specific TLV "Maximum Frame Size" (OUI 00-12-0F, subtype 4):
    // the largest frame the switch port accepts, Ethernet header and FCS included (1518 for a
    // 1500-byte MTU, e.g. 9216 on a jumbo port).  nullopt when the switch does not send it.
    std::optional<uint16_t> max_frame_size() const;
    void set_max_frame_size(uint16_t bytes);
};

enum class DecodeError {
    None = 0,
    TooShort,
    NotLldp,
    TlvOverrun,
    MissingChassisId,
    MissingPortId,
    MissingTtl,
    BadChassisId,
    BadPortId,
    BadTtl,
    BadManagementAddress,
    BadOrgTlv,
    DuplicateMandatory,
};
const char* to_string(DecodeError e);

// Decodes an Ethernet frame (starting at the destination MAC) carrying an LLDPDU.
std::optional<Frame> decode(const uint8_t* data, size_t len, DecodeError* err = nullptr);
inline std::optional<Frame> decode(const std::string& bytes, DecodeError* err = nullptr) {
    return decode(reinterpret_cast<const uint8_t*>(bytes.data()), bytes.size(), err);
}

// Encodes a full Ethernet frame (padded to the 60-byte minimum).
std::vector<uint8_t> encode(const Frame& f);

// Convenience: a switch-port LLDPDU as a ToR switch would send it.
Frame make_switch_frame(const MacAddr& switch_port_mac, const std::string& system_name,
                        const std::string& port_name, const std::string& port_description, uint16_t ttl = 120);

}  // namespace netop::lldp
