#include "netop/lldp.hpp"

#include <algorithm>

namespace netop::lldp {

const MacAddr kNearestBridge{{0x01, 0x80, 0xc2, 0x00, 0x00, 0x0e}};
const MacAddr kNearestNonTpmrBridge{{0x01, 0x80, 0xc2, 0x00, 0x00, 0x03}};
const MacAddr kNearestCustomerBridge{{0x01, 0x80, 0xc2, 0x00, 0x00, 0x00}};

const char* to_string(DecodeError e) {
    switch (e) {
        case DecodeError::None: return "ok";
        case DecodeError::TooShort: return "frame too short";
        case DecodeError::NotLldp: return "not an LLDP ethertype";
        case DecodeError::TlvOverrun: return "TLV length overruns frame";
        case DecodeError::MissingChassisId: return "first TLV is not Chassis ID";
        case DecodeError::MissingPortId: return "second TLV is not Port ID";
        case DecodeError::MissingTtl: return "third TLV is not TTL";
        case DecodeError::BadChassisId: return "malformed Chassis ID TLV";
        case DecodeError::BadPortId: return "malformed Port ID TLV";
        case DecodeError::BadTtl: return "malformed TTL TLV";
        case DecodeError::BadManagementAddress: return "malformed Management Address TLV";
        case DecodeError::BadOrgTlv: return "malformed organizationally specific TLV";
        case DecodeError::DuplicateMandatory: return "duplicate mandatory TLV";
    }
    return "unknown";
}

std::optional<MacAddr> Frame::peer_mac() const {
    std::optional<MacAddr> m;
    if (chassis_subtype == kChassisMac && chassis_id.size() == 6)
        m = MacAddr::from_bytes(reinterpret_cast<const uint8_t*>(chassis_id.data()));
    if (port_subtype == kPortMac && port_id.size() == 6)
        m = MacAddr::from_bytes(reinterpret_cast<const uint8_t*>(port_id.data()));
    return m;
}

static std::string id_str(bool is_mac, const std::string& raw) {
    if (is_mac && raw.size() == 6) return MacAddr::from_bytes(reinterpret_cast<const uint8_t*>(raw.data())).str();
    return raw;
}

std::string Frame::chassis_id_str() const { return id_str(chassis_subtype == kChassisMac, chassis_id); }
std::string Frame::port_id_str() const { return id_str(port_subtype == kPortMac, port_id); }

static inline uint16_t be16(const uint8_t* p) { return uint16_t(p[0] << 8 | p[1]); }

std::optional<Frame> decode(const uint8_t* p, size_t len, DecodeError* err) {
    DecodeError dummy;
    DecodeError& e = err ? *err : dummy;
    e = DecodeError::None;
    if (len < 14) {
        e = DecodeError::TooShort;
        return std::nullopt;
    }
    Frame f;
    f.dst = MacAddr::from_bytes(p);
    f.src = MacAddr::from_bytes(p + 6);
    size_t off = 12;
    uint16_t et = be16(p + off);
    // Strip up to two VLAN tags (802.1Q / 802.1ad) left in the frame.
    for (int tags = 0; (et == 0x8100 || et == 0x88a8) && tags < 2; ++tags) {
        if (len < off + 6) {
            e = DecodeError::TooShort;
            return std::nullopt;
        }
        f.vlan = uint16_t(be16(p + off + 2) & 0x0fff);
        off += 4;
        et = be16(p + off);
    }
    if (et != kEtherType) {
        e = DecodeError::NotLldp;
        return std::nullopt;
    }
    off += 2;

    int index = 0;
    bool have_ttl = false;
    while (off + 2 <= len) {
        uint16_t hdr = be16(p + off);
        uint8_t type = uint8_t(hdr >> 9);
        size_t tlen = hdr & 0x1ff;
        off += 2;
        if (off + tlen > len) {
            e = DecodeError::TlvOverrun;
            return std::nullopt;
        }
        const uint8_t* v = p + off;
        off += tlen;

        // Mandatory order: Chassis ID, Port ID, TTL (IEEE 802.1AB-2016 §8.2).
        if (index == 0 && type != kChassisId) {
            e = DecodeError::MissingChassisId;
            return std::nullopt;
        }
        if (index == 1 && type != kPortId) {
            e = DecodeError::MissingPortId;
            return std::nullopt;
        }
        if (index == 2 && type != kTtl) {
            e = DecodeError::MissingTtl;
            return std::nullopt;
        }
        ++index;
        if (type == kEnd) break;

        switch (type) {
            case kChassisId:
                if (index != 1) {
                    e = DecodeError::DuplicateMandatory;
                    return std::nullopt;
                }
                if (tlen < 2) {
                    e = DecodeError::BadChassisId;
                    return std::nullopt;
                }
                f.chassis_subtype = v[0];
                f.chassis_id.assign(reinterpret_cast<const char*>(v + 1), tlen - 1);
                break;
            case kPortId:
                if (index != 2) {
                    e = DecodeError::DuplicateMandatory;
                    return std::nullopt;
                }
                if (tlen < 2) {
                    e = DecodeError::BadPortId;
                    return std::nullopt;
                }
                f.port_subtype = v[0];
                f.port_id.assign(reinterpret_cast<const char*>(v + 1), tlen - 1);
                break;
            case kTtl:
                if (index != 3) {
                    e = DecodeError::DuplicateMandatory;
                    return std::nullopt;
                }
                if (tlen < 2) {
                    e = DecodeError::BadTtl;
                    return std::nullopt;
                }
                f.ttl = be16(v);
                have_ttl = true;
                break;
            case kPortDescription:
                f.port_description.emplace(reinterpret_cast<const char*>(v), tlen);
                break;
            case kSystemName:
                f.system_name.emplace(reinterpret_cast<const char*>(v), tlen);
                break;
            case kSystemDescription:
                f.system_description.emplace(reinterpret_cast<const char*>(v), tlen);
                break;
            case kSystemCapabilities:
                if (tlen >= 4) f.capabilities = std::make_pair(be16(v), be16(v + 2));
                break;
            case kManagementAddress: {
                // addr-string-len(1) = 1 + |addr|; subtype(1); addr; if-subtype(1); if-num(4); oid-len(1); oid
                if (tlen < 9) {
                    e = DecodeError::BadManagementAddress;
                    return std::nullopt;
                }
                size_t alen = v[0];
                if (alen < 2 || alen > 32 || 1 + alen + 5 + 1 > tlen) {
                    e = DecodeError::BadManagementAddress;
                    return std::nullopt;
                }
                ManagementAddress m;
                m.addr_subtype = v[1];
                m.address.assign(reinterpret_cast<const char*>(v + 2), alen - 1);
                size_t q = 1 + alen;
                m.if_subtype = v[q];
                m.if_number = uint32_t(v[q + 1]) << 24 | uint32_t(v[q + 2]) << 16 | uint32_t(v[q + 3]) << 8 | v[q + 4];
                size_t olen = v[q + 5];
                if (q + 6 + olen > tlen) {
                    e = DecodeError::BadManagementAddress;
                    return std::nullopt;
                }
                m.oid.assign(reinterpret_cast<const char*>(v + q + 6), olen);
                f.management.push_back(std::move(m));
                break;
            }
            case kOrgSpecific: {
                if (tlen < 4) {
                    e = DecodeError::BadOrgTlv;
                    return std::nullopt;
                }
                OrgTlv o;
                o.oui = uint32_t(v[0]) << 16 | uint32_t(v[1]) << 8 | v[2];
                o.subtype = v[3];
                o.info.assign(reinterpret_cast<const char*>(v + 4), tlen - 4);
                f.org.push_back(std::move(o));
                break;
            }
            default:
                break;  // reserved types: skip
        }
    }
    if (index == 0) {
        e = DecodeError::MissingChassisId;
        return std::nullopt;
    }
    if (index == 1) {
        e = DecodeError::MissingPortId;
        return std::nullopt;
    }
    if (!have_ttl) {
        e = DecodeError::MissingTtl;
        return std::nullopt;
    }
    return f;
}

static void put_tlv(std::vector<uint8_t>& out, uint8_t type, const std::string& value) {
    size_t n = value.size() > 511 ? 511 : value.size();
    out.push_back(uint8_t(type << 1 | ((n >> 8) & 1)));
    out.push_back(uint8_t(n & 0xff));
    out.insert(out.end(), value.begin(), value.begin() + long(n));
}

std::vector<uint8_t> encode(const Frame& f) {
    std::vector<uint8_t> out;
    out.reserve(128);
    out.insert(out.end(), f.dst.b.begin(), f.dst.b.end());
    out.insert(out.end(), f.src.b.begin(), f.src.b.end());
    if (f.vlan) {
        out.push_back(0x81);
        out.push_back(0x00);
        out.push_back(uint8_t((*f.vlan >> 8) & 0x0f));
        out.push_back(uint8_t(*f.vlan & 0xff));
    }
    out.push_back(uint8_t(kEtherType >> 8));
    out.push_back(uint8_t(kEtherType & 0xff));
    put_tlv(out, kChassisId, std::string(1, char(f.chassis_subtype)) + f.chassis_id.substr(0, 255));
    put_tlv(out, kPortId, std::string(1, char(f.port_subtype)) + f.port_id.substr(0, 255));
    put_tlv(out, kTtl, std::string{char(f.ttl >> 8), char(f.ttl & 0xff)});
    if (f.port_description) put_tlv(out, kPortDescription, *f.port_description);
    if (f.system_name) put_tlv(out, kSystemName, *f.system_name);
    if (f.system_description) put_tlv(out, kSystemDescription, *f.system_description);
    if (f.capabilities) {
        auto [a, b] = *f.capabilities;
        put_tlv(out, kSystemCapabilities, std::string{char(a >> 8), char(a), char(b >> 8), char(b)});
    }
    for (const auto& m : f.management) {
        std::string v;
        v.push_back(char(1 + m.address.size()));
        v.push_back(char(m.addr_subtype));
        v += m.address;
        v.push_back(char(m.if_subtype));
        v.push_back(char(m.if_number >> 24));
        v.push_back(char(m.if_number >> 16));
        v.push_back(char(m.if_number >> 8));
        v.push_back(char(m.if_number));
        v.push_back(char(m.oid.size()));
        v += m.oid;
        put_tlv(out, kManagementAddress, v);
    }
    for (const auto& o : f.org) {
        std::string v{char(o.oui >> 16), char(o.oui >> 8), char(o.oui), char(o.subtype)};
        v += o.info;
        put_tlv(out, kOrgSpecific, v);
    }
    out.push_back(0);  // End of LLDPDU
    out.push_back(0);
    if (out.size() < 60) out.resize(60, 0);
    return out;
}

constexpr uint32_t kOui8023 = 0x00120F;
constexpr uint8_t kMaxFrameSizeSubtype = 4;

std::optional<uint16_t> Frame::max_frame_size() const {
    for (const auto& o : org)
        if (o.oui == kOui8023 && o.subtype == kMaxFrameSizeSubtype && o.info.size() == 2)
            return uint16_t((uint8_t(o.info[0]) << 8) | uint8_t(o.info[1]));
    return std::nullopt;
}

void Frame::set_max_frame_size(uint16_t bytes) {
    org.erase(std::remove_if(org.begin(), org.end(),
                             [](const OrgTlv& o) { return o.oui == kOui8023 && o.subtype == kMaxFrameSizeSubtype; }),
              org.end());
    org.push_back(OrgTlv{kOui8023, kMaxFrameSizeSubtype, std::string{char(bytes >> 8), char(bytes & 0xff)}});
}

Frame make_switch_frame(const MacAddr& switch_port_mac, const std::string& system_name, const std::string& port_name,
                        const std::string& port_description, uint16_t ttl) {
    Frame f;
    f.dst = kNearestBridge;
    f.src = switch_port_mac;
    f.chassis_subtype = kChassisMac;
    f.chassis_id.assign(reinterpret_cast<const char*>(switch_port_mac.b.data()), 6);
    f.port_subtype = kPortIfName;
    f.port_id = port_name;
    f.ttl = ttl;
    f.port_description = port_description;
    f.system_name = system_name;
    f.system_description = "synthetic ToR switch (amd network-operator harness)";
    f.capabilities = std::make_pair(uint16_t(0x0014), uint16_t(0x0014));  // bridge + router
    return f;
}

}  // namespace netop::lldp
