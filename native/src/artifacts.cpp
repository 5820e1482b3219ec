#include "netop/artifacts.hpp"

#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <set>

#include "netop/log.hpp"

namespace netop::artifacts {

// ---------------------------------------------------------------------------
// Json
// ---------------------------------------------------------------------------
std::string Json::escape(const std::string& s) {
    std::string o;
    o.reserve(s.size() + 2);
    for (unsigned char c : s) {
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break;
            case '\t': o += "\\t"; break;
            case '<': o += "\\u003c"; break;  // Go's HTML-safe escaping
            case '>': o += "\\u003e"; break;
            case '&': o += "\\u0026"; break;
            default:
                if (c < 0x20)
                    o += strfmt("\\u%04x", c);
                else
                    o += char(c);
        }
    }
    return o;
}

void Json::sep() {
    if (after_key_) {
        after_key_ = false;
        return;
    }
    if (!first_.back()) out_ += ',';
    first_.back() = false;
}
Json& Json::begin_object() {
    sep();
    out_ += '{';
    first_.push_back(true);
    return *this;
}
Json& Json::end_object() {
    out_ += '}';
    first_.pop_back();
    return *this;
}
Json& Json::begin_array() {
    sep();
    out_ += '[';
    first_.push_back(true);
    return *this;
}
Json& Json::end_array() {
    out_ += ']';
    first_.pop_back();
    return *this;
}
Json& Json::key(const std::string& k) {
    sep();
    out_ += '"' + escape(k) + "\":";
    after_key_ = true;
    return *this;
}
Json& Json::value(const std::string& s) {
    sep();
    out_ += '"' + escape(s) + '"';
    return *this;
}
Json& Json::value(int64_t v) {
    sep();
    out_ += std::to_string(v);
    return *this;
}
Json& Json::value(uint64_t v) {
    sep();
    out_ += std::to_string(v);
    return *this;
}
Json& Json::value(double v) {
    sep();
    if (!std::isfinite(v))
        out_ += "null";
    else
        out_ += strfmt("%.9g", v);
    return *this;
}
Json& Json::value(bool b) {
    sep();
    out_ += b ? "true" : "false";
    return *this;
}
Json& Json::null() {
    sep();
    out_ += "null";
    return *this;
}

// ---------------------------------------------------------------------------
// RCCL artifacts
// ---------------------------------------------------------------------------
static std::vector<const NicState*> sorted(const std::vector<NicState>& nics) {
    std::vector<const NicState*> v;
    for (auto& n : nics) v.push_back(&n);
    std::stable_sort(v.begin(), v.end(), [](const NicState* a, const NicState* b) {
        int ga = a->gpu_index < 0 ? 1 << 30 : a->gpu_index, gb = b->gpu_index < 0 ? 1 << 30 : b->gpu_index;
        return ga != gb ? ga < gb : a->ifname < b->ifname;
    });
    return v;
}

std::string generate_rccl_net(const std::vector<NicState>& nics, bool extended) {
    Json j;
    j.begin_object().key("NIC_NET_CONFIG").begin_array();
    for (const NicState* n : sorted(nics)) {
        if (!n->addr) {
            NLOG_W("Interface '%s' has no LLDP address when creating RCCL network file, skipping...", n->ifname.c_str());
            continue;
        }
        if (!n->peer_mac) {
            NLOG_W("Interface '%s' has no peer MAC address when creating RCCL network file, skipping...", n->ifname.c_str());
            continue;
        }
        j.begin_object();
        j.key("NIC_MAC").value(n->link.mac.str());
        j.key("NIC_IP").value(n->addr->local.str());
        j.key("SUBNET_MASK").value(l3::mask_string(n->addr->prefix));
        j.key("GATEWAY_MAC").value(n->peer_mac->str());
        if (extended) {
            j.key("NIC_NAME").value(n->ifname);
            j.key("GATEWAY_IP").value(n->addr->peer.str());
            if (!n->gpu_bdf.empty()) j.key("GPU_BDF").value(n->gpu_bdf);
            if (n->gpu_index >= 0) j.key("GPU_INDEX").value(n->gpu_index);
            if (!n->rdma_dev.empty()) {
                j.key("RDMA_DEV").value(n->rdma_dev);
                j.key("RDMA_PORT").value(n->rdma_port);
            }
            if (n->gid_index) j.key("GID_INDEX").value(*n->gid_index);
            if (n->numa_node >= 0) j.key("NUMA_NODE").value(n->numa_node);
            if (!n->pcie_path.empty()) j.key("PCIE_PATH").value(n->pcie_path);
        }
        j.end_object();
    }
    j.end_array().end_object();
    return j.str();
}

void write_rccl_net(const std::string& path, const std::vector<NicState>& nics, bool extended) {
    if (path.empty()) throw std::runtime_error("no file name when saving the RCCL network file");
    write_file_atomic(path, generate_rccl_net(nics, extended), 0644);
}

std::vector<std::pair<std::string, std::string>> parse_env_extra(const std::string& spec) {
    std::vector<std::pair<std::string, std::string>> out;
    for (const auto& item : split(spec, ',')) {
        std::string t = trim(item);
        if (t.empty()) continue;
        auto eq = t.find('=');
        if (eq == std::string::npos) throw std::invalid_argument("bad RCCL env entry '" + t + "' (want KEY=VALUE)");
        std::string k = t.substr(0, eq), v = t.substr(eq + 1);
        bool prefix = k.rfind("NCCL_", 0) == 0 || k.rfind("RCCL_", 0) == 0 || k.rfind("HSA_", 0) == 0;
        bool chars = !k.empty() && std::all_of(k.begin(), k.end(), [](char c) {
            return (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
        });
        if (!prefix || !chars) throw std::invalid_argument("RCCL env key '" + k + "' must be NCCL_*, RCCL_* or HSA_*");
        if (v.find_first_of("\n\r") != std::string::npos) throw std::invalid_argument("multi-line value for " + k);
        out.emplace_back(k, v);
    }
    return out;
}

std::string generate_rccl_env(const std::vector<NicState>& nics, const std::string& topo_file,
                              const std::vector<std::pair<std::string, std::string>>& extra,
                              const std::vector<std::string>& socket_ifnames, bool link_local) {
    std::vector<std::string> hcas;
    std::set<int> gids;
    bool gid_unknown = false;
    for (const NicState* n : sorted(nics)) {
        if (n->rdma_dev.empty() || !n->configured) continue;
        hcas.push_back(n->rdma_dev + ":" + std::to_string(n->rdma_port));
        if (n->gid_index)
            gids.insert(*n->gid_index);
        else
            gid_unknown = true;
    }
    std::string out = "# Generated by the AMD network operator link-discovery agent.\n"
                      "# Source this file (or pass it as an env-file) in RCCL jobs on this node.\n";
    if (!hcas.empty()) out += "NCCL_IB_HCA==" + join(hcas, ",") + "\n";
    if (gids.size() == 1 && !gid_unknown) {
        out += "NCCL_IB_GID_INDEX=" + std::to_string(*gids.begin()) + "\n";
    } else if (!hcas.empty()) {
        out += "NCCL_IB_ROCE_VERSION_NUM=2\n";
        out += std::string("NCCL_IB_ADDR_FAMILY=") + (link_local ? "AF_INET6" : "AF_INET") + "\n";
    }
    if (!hcas.empty()) out += "NCCL_IB_DISABLE=0\n";
    if (!socket_ifnames.empty()) out += "NCCL_SOCKET_IFNAME==" + join(socket_ifnames, ",") + "\n";
    if (!topo_file.empty()) out += "NCCL_TOPO_FILE=" + topo_file + "\n";
    for (auto& [k, v] : extra) out += k + "=" + v + "\n";
    return out;
}

void write_rccl_env(const std::string& path, const std::vector<NicState>& nics, const std::string& topo_file,
                    const std::vector<std::pair<std::string, std::string>>& extra,
                    const std::vector<std::string>& socket_ifnames, bool link_local) {
    write_file_atomic(path, generate_rccl_env(nics, topo_file, extra, socket_ifnames, link_local), 0644);
}

// ---------------------------------------------------------------------------
// NCCL_TOPO_FILE
// ---------------------------------------------------------------------------
namespace {
struct XmlPci {
    topo::PciDev dev;
    std::vector<std::unique_ptr<XmlPci>> kids;
    std::vector<const TopoNic*> nets;
};

XmlPci& child(std::vector<std::unique_ptr<XmlPci>>& level, const topo::PciDev& d) {
    for (auto& k : level)
        if (k->dev.bdf == d.bdf) return *k;
    level.push_back(std::make_unique<XmlPci>());
    level.back()->dev = d;
    return *level.back();
}

std::string xml_attr(const std::string& s) {
    std::string o;
    for (char c : s) {
        switch (c) {
            case '"': o += "&quot;"; break;
            case '&': o += "&amp;"; break;
            case '<': o += "&lt;"; break;
            case '>': o += "&gt;"; break;
            default: o += c;
        }
    }
    return o;
}

void emit_pci(std::string& out, XmlPci& n, int depth) {
    std::sort(n.kids.begin(), n.kids.end(), [](const auto& a, const auto& b) { return a->dev.bdf < b->dev.bdf; });
    const std::string ind(size_t(depth) * 2, ' ');
    const auto& d = n.dev;
    out += ind + "<pci busid=\"" + xml_attr(d.bdf) + "\"";
    if (d.pci_class) out += strfmt(" class=\"0x%06x\"", d.pci_class);
    if (d.vendor) out += strfmt(" vendor=\"0x%04x\"", d.vendor);
    if (d.device) out += strfmt(" device=\"0x%04x\"", d.device);
    if (d.subsystem_vendor) out += strfmt(" subsystem_vendor=\"0x%04x\"", d.subsystem_vendor);
    if (d.subsystem_device) out += strfmt(" subsystem_device=\"0x%04x\"", d.subsystem_device);
    // Always written: RCCL fills link attributes only on the PCI nodes it walks up from a GPU,
    // not on a NIC's node that it finds in the file by name, and refuses a node without them
    // ("Attribute link_width of node pci not found", measured on the box).
    out += " link_speed=\"" + xml_attr(d.rccl_link_speed()) + "\"";
    out += strfmt(" link_width=\"%d\"", d.rccl_link_width());
    if (n.kids.empty() && n.nets.empty()) {
        out += "/>\n";
        return;
    }
    out += ">\n";
    for (auto& k : n.kids) emit_pci(out, *k, depth + 1);
    if (!n.nets.empty()) {
        out += ind + "  <nic>\n";
        for (const TopoNic* t : n.nets) {
            out += ind + "    <net name=\"" + xml_attr(t->net_name) + "\"";
            if (t->port > 0) out += strfmt(" port=\"%d\"", t->port);
            out += "/>\n";
        }
        out += ind + "  </nic>\n";
    }
    out += ind + "</pci>\n";
}
}  // namespace

std::string generate_rccl_topo(const std::vector<topo::Gpu>& gpus, const std::vector<TopoNic>& nics,
                               const topo::CpuIdentity& cpu, const std::string& sysfs_root, int version) {
    std::map<int, std::vector<std::unique_ptr<XmlPci>>> cpus;  // numaid -> top-level PCI nodes
    std::map<std::string, topo::PciDev> bridges;
    auto place = [&](const topo::PciDev& found) -> XmlPci& {
        std::optional<topo::PciDev> full;  // discovery reads devices without the topology attributes
        if (!found.topo_attrs) {
            full = found;
            topo::read_topo_attrs(*full);
        }
        const topo::PciDev& leaf = full ? *full : found;
        auto parents = topo::rccl_pci_parents(leaf, &bridges);
        auto* level = &cpus[parents.empty() ? leaf.numa : parents.front().numa];
        for (const auto& p : parents) level = &child(*level, p).kids;
        return child(*level, leaf);
    };
    for (const auto& g : gpus) place(g.pci);
    for (const auto& n : nics) {
        if (n.net_name.empty() || n.pci.bdf.empty()) continue;
        place(n.pci).nets.push_back(&n);
    }
    std::string out = strfmt("<system version=\"%d\">\n", version);
    for (auto& [numa, tops] : cpus) {
        out += strfmt("  <cpu numaid=\"%d\"", numa);
        const std::string aff = topo::numa_cpumap(sysfs_root, numa);
        if (!aff.empty()) out += " affinity=\"" + xml_attr(aff) + "\"";
        if (!cpu.arch.empty()) out += " arch=\"" + xml_attr(cpu.arch) + "\"";
        if (!cpu.vendor.empty()) out += " vendor=\"" + xml_attr(cpu.vendor) + "\"";
        if (cpu.family >= 0) out += strfmt(" familyid=\"%d\"", cpu.family);
        if (cpu.model >= 0) out += strfmt(" modelid=\"%d\"", cpu.model);
        out += ">\n";
        std::sort(tops.begin(), tops.end(), [](const auto& a, const auto& b) { return a->dev.bdf < b->dev.bdf; });
        for (auto& t : tops) emit_pci(out, *t, 2);
        out += "  </cpu>\n";
    }
    out += "</system>\n";
    return out;
}

void write_rccl_topo(const std::string& path, const std::vector<topo::Gpu>& gpus, const std::vector<TopoNic>& nics,
                     const topo::CpuIdentity& cpu, const std::string& sysfs_root, int version) {
    write_file_atomic(path, generate_rccl_topo(gpus, nics, cpu, sysfs_root, version), 0644);
}

std::vector<TopoNic> topo_nics(const topo::DiscoveryResult& d, const std::vector<std::string>& names,
                               const std::string& sysfs_root) {
    std::vector<TopoNic> out;
    for (const auto& name : names) {
        TopoNic t;
        bool found = false;
        for (const auto& n : d.nics) {
            if (n.ifname != name) continue;
            t.pci = n.pci;
            t.net_name = n.rdma_dev.empty() ? n.ifname : n.rdma_dev;
            t.port = n.rdma_dev.empty() ? 0 : n.rdma_port;
            found = true;
            break;
        }
        if (!found) {
            auto p = topo::netdev_pci(sysfs_root, name);
            if (!p) continue;  // virtual link: nothing PCIe to pin
            t.pci = *p;
            auto ib = list_dir(path_join(p->path, "infiniband"));
            t.net_name = ib.empty() ? name : ib.front();
            if (!ib.empty()) {
                auto port = read_file(path_join(sysfs_root, "class/net/" + name + "/dev_port"));
                t.port = (port ? std::atoi(trim(*port).c_str()) : 0) + 1;
            }
        }
        out.push_back(std::move(t));
    }
    return out;
}

// ---------------------------------------------------------------------------
// systemd-networkd
// ---------------------------------------------------------------------------
std::string networkd_filename(const std::string& dir, const std::string& ifname) {
    return path_join(dir, ifname + ".network");
}

std::string generate_networkd(const NicState& n) {
    Ipv4Prefix routed = n.addr->routed_network();
    return strfmt(
        "[Match]\n"
        "MACAddress=%s\n"
        "\n"
        "[Network]\n"
        "Description=Networkd configuration for %s created by network-operator\n"
        "Address=%s/%d\n"
        "\n"
        "[Route]\n"
        "Destination=%s/%d\n",
        n.link.mac.str().c_str(), n.ifname.c_str(), n.addr->local.str().c_str(), n.addr->prefix,
        routed.addr.str().c_str(), routed.len);
}

std::vector<std::string> write_networkd(const std::string& dir, const std::vector<NicState>& nics) {
    for (auto& n : nics) {
        if (n.link.index == 0 && n.link.name.empty()) throw std::runtime_error("no link information for " + n.ifname);
        if (!n.addr) throw std::runtime_error("no local address for " + n.ifname);
        if (n.link.mac.is_zero()) throw std::runtime_error("no local hw address for " + n.ifname);
    }
    std::vector<std::string> written;
    for (const NicState* n : sorted(nics)) {
        std::string fn = networkd_filename(dir, n->ifname);
        try {
            write_file_atomic(fn, generate_networkd(*n), 0644);
        } catch (const std::exception& e) {
            delete_networkd(dir, written);
            throw std::runtime_error("could not write networkd config file '" + fn + "': " + e.what());
        }
        written.push_back(n->ifname);
    }
    return written;
}

void delete_networkd(const std::string& dir, const std::vector<std::string>& ifnames) {
    for (auto& i : ifnames) ::unlink(networkd_filename(dir, i).c_str());
}

// ---------------------------------------------------------------------------
// NFD labels
// ---------------------------------------------------------------------------
const char* const kScaleOutReadyLabel = "amd.feature.node.kubernetes.io/gpu-scale-out=true";

std::string Labels::path() const { return path_join(dir, file); }

std::string generate_labels(const std::map<std::string, std::string>& extra, const std::string& key) {
    std::string out = key + "=true\n";
    for (auto& [k, v] : extra) out += k + "=" + v + "\n";
    return out;
}

bool write_labels(const Labels& l, const std::map<std::string, std::string>& extra) {
    if (!is_dir(l.dir)) return false;
    write_file_atomic(l.path(), generate_labels(extra, l.key), 0644);
    return true;
}

bool remove_labels(const Labels& l) { return ::unlink(l.path().c_str()) == 0; }

// ---------------------------------------------------------------------------
// LLDP cache
// ---------------------------------------------------------------------------
static const char* const kLldpCacheHeader = "# netop-lldp-cache v1";

static std::string one_field(const std::string& s) {
    std::string o = s;
    for (char& c : o)
        if (c == '\t' || c == '\n' || c == '\r') c = ' ';
    return o.empty() ? "-" : o;
}

std::vector<LldpCacheEntry> read_lldp_cache(const std::string& path) {
    auto text = read_file(path);
    return text ? decode_lldp_cache(*text) : std::vector<LldpCacheEntry>{};
}

std::vector<LldpCacheEntry> decode_lldp_cache(const std::string& text) {
    std::vector<LldpCacheEntry> out;
    auto lines = split(text, '\n');
    if (lines.empty() || trim(lines[0]) != kLldpCacheHeader) return out;  // unknown format: ignore
    for (size_t i = 1; i < lines.size(); ++i) {
        auto f = split(lines[i], '\t');
        if (f.size() != 7) continue;
        LldpCacheEntry e;
        e.nic_mac = f[0];
        e.ifname = f[1];
        e.unix_s = std::strtoll(f[2].c_str(), nullptr, 10);
        e.peer_mac = f[3] == "-" ? "" : f[3];
        e.system_name = f[4] == "-" ? "" : f[4];
        e.port_id = f[5] == "-" ? "" : f[5];
        e.port_description = f[6] == "-" ? "" : f[6];
        out.push_back(std::move(e));
    }
    return out;
}

std::string encode_lldp_cache(const std::vector<LldpCacheEntry>& entries) {
    std::string out = std::string(kLldpCacheHeader) + "\n";
    for (const auto& e : entries)
        out += one_field(e.nic_mac) + "\t" + one_field(e.ifname) + "\t" + std::to_string(e.unix_s) + "\t" +
               one_field(e.peer_mac) + "\t" + one_field(e.system_name) + "\t" + one_field(e.port_id) + "\t" +
               one_field(e.port_description) + "\n";
    return out;
}

void write_lldp_cache(const std::string& path, const std::vector<LldpCacheEntry>& entries) {
    write_file_atomic(path, encode_lldp_cache(entries), 0644);
}

// ---------------------------------------------------------------------------
// Status document
// ---------------------------------------------------------------------------
std::string generate_status(const std::vector<NicState>& nics, const std::map<std::string, int64_t>& phases_ns,
                            int64_t t0, const std::string& mode, bool ready,
                            const std::map<std::string, std::string>& node) {
    Json j;
    j.begin_object();
    j.key("mode").value(mode);
    j.key("ready").value(ready);
    for (auto& [k, v] : node) j.key(k).value(v);
    j.key("phases_ms").begin_object();
    for (auto& [k, v] : phases_ns) j.key(k).value(double(v) / 1e6);
    j.end_object();
    j.key("interfaces").begin_array();
    for (const NicState* n : sorted(nics)) {
        j.begin_object();
        j.key("name").value(n->ifname);
        j.key("mac").value(n->link.mac.str());
        j.key("gpu_index").value(n->gpu_index);
        if (!n->gpu_bdf.empty()) j.key("gpu_bdf").value(n->gpu_bdf);
        if (!n->rdma_dev.empty()) j.key("rdma_dev").value(n->rdma_dev);
        if (!n->fw_lldp.empty()) j.key("fw_lldp").value(n->fw_lldp);
        if (!n->dcbx.empty()) j.key("dcbx").value(n->dcbx);
        if (!n->driver.empty()) j.key("driver").value(n->driver);
        if (!n->lldp_silent.empty()) j.key("lldp_silent").value(n->lldp_silent);
        if (n->speed_mbps >= 0) j.key("speed_mbps").value(n->speed_mbps);
        if (n->pcie.known()) j.key("pcie").value(n->pcie.str());
        if (n->gpu_pcie.known()) j.key("gpu_pcie").value(n->gpu_pcie.str());
        if (n->peer_max_frame > 0) j.key("peer_max_frame").value(n->peer_max_frame);
        j.key("lldp").value(n->lldp_seen);
        if (n->lldp_seen) {
            j.key("lldp_source").value(n->lldp_from_cache ? "cache" : "frame");
            if (n->cache_stale) j.key("cache_unconfirmed").value(true);
            j.key("port_description").value(n->port_description);
            if (n->peer_mac) j.key("peer_mac").value(n->peer_mac->str());
            j.key("peer_system").value(n->peer_system_name);
        }
        if (n->addr) {
            j.key("local").value(n->addr->local_prefix().str());
            j.key("gateway").value(n->addr->peer.str());
        }
        if (!n->addr_error.empty()) j.key("addr_error").value(n->addr_error);
        j.key("configured").value(n->configured);
        if (n->awaiting_carrier) j.key("awaiting_carrier").value(true);
        if (n->no_carrier) j.key("no_carrier").value(true);
        j.key("degraded").value(n->degraded);
        if (n->flaps) j.key("flaps").value(n->flaps);
        if (!n->config_error.empty()) j.key("config_error").value(n->config_error);
        if (n->peer_verified) {
            j.key("peer_verified").value(true);
            j.key("peer_arp_ms").value(double(n->peer_rtt_ns) / 1e6);
            j.key("peer_verify_ms").value(double(n->peer_verify_ns) / 1e6);
            if (n->peer_arp_mac) j.key("peer_arp_mac").value(n->peer_arp_mac->str());
            if (n->peer_mac_mismatch) j.key("peer_mac_mismatch").value(true);
        }
        if (!n->peer_error.empty()) j.key("peer_error").value(n->peer_error);
        if (n->gid_index) j.key("gid_index").value(*n->gid_index);
        if (n->t_lldp) j.key("t_lldp_ms").value(double(n->t_lldp - t0) / 1e6);
        if (n->t_configured) j.key("t_configured_ms").value(double(n->t_configured - t0) / 1e6);
        j.end_object();
    }
    j.end_array();
    j.end_object();
    return j.str();
}

}  // namespace netop::artifacts
