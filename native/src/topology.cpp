#include "netop/topology.hpp"

#include "netop/bounded.hpp"

#include <fcntl.h>
#include <sys/utsname.h>
#include <unistd.h>
#include <cerrno>
#include <climits>
#if defined(__x86_64__)
#include <cpuid.h>
#endif

#include <algorithm>
#include <cstdlib>
#include <cfloat>
#include <cstdio>
#include <cstring>
#include <set>

#include "netop/log.hpp"

namespace netop::topo {

std::string sysfs_root() {
    const char* r = std::getenv("SYSFS_ROOT");
    return (r && *r) ? std::string(r) : std::string("/sys/");
}

const char* to_string(PathType p) {
    switch (p) {
        case PathType::PIX: return "PIX";
        case PathType::PXB: return "PXB";
        case PathType::PHB: return "PHB";
        case PathType::NODE: return "NODE";
        case PathType::SYS: return "SYS";
    }
    return "SYS";
}

std::optional<DiscoveryMode> parse_discovery_mode(std::string_view s) {
    if (s == "affine" || s.empty()) return DiscoveryMode::Affine;
    if (s == "accel") return DiscoveryMode::Accel;
    if (s == "rdma") return DiscoveryMode::Rdma;
    if (s == "none") return DiscoveryMode::None;
    return std::nullopt;
}

static bool looks_like_bdf(std::string_view s) {
    // dddd:bb:dd.f
    if (s.size() != 12) return false;
    auto hex = [](char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); };
    for (size_t i = 0; i < 12; ++i) {
        if (i == 4 || i == 7) {
            if (s[i] != ':') return false;
        } else if (i == 10) {
            if (s[i] != '.') return false;
        } else if (!hex(s[i])) {
            return false;
        }
    }
    return true;
}

// A sysfs attribute: at most a page, returned by a single read().  `dirfd` (optional) is an
// open directory the name is relative to: a device's attributes are then looked up one
// component deep instead of walking the whole sysfs path again for each of them.
static std::optional<std::string> read_attr(const std::string& path, int dirfd = AT_FDCWD) {
    int fd = ::openat(dirfd, path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return std::nullopt;
    char buf[4096];
    ssize_t n;
    do {
        n = ::read(fd, buf, sizeof buf);
    } while (n < 0 && errno == EINTR);
    ::close(fd);
    if (n < 0) return std::nullopt;
    return std::string(buf, size_t(n));
}

static uint32_t read_hex(const std::string& path, int dirfd = AT_FDCWD) {
    auto s = read_attr(path, dirfd);
    if (!s) return 0;
    return uint32_t(std::strtoul(trim(*s).c_str(), nullptr, 16));
}

static int read_int(const std::string& path, int dflt, int dirfd = AT_FDCWD) {
    auto s = read_attr(path, dirfd);
    if (!s) return dflt;
    auto t = trim(*s);
    if (t.empty()) return dflt;
    return int(std::strtol(t.c_str(), nullptr, 10));
}

std::optional<PciDev> read_pci_dev(const std::string& root, const std::string& device_path, bool topo_attrs) {
    (void)root;
    auto real = realpath_of(device_path);
    if (!real) return std::nullopt;
    return read_pci_dir(*real, topo_attrs);
}

static void topo_attrs_at(int dir, PciDev& d) {
    d.topo_attrs = true;
    d.subsystem_vendor = read_hex("subsystem_vendor", dir);
    d.subsystem_device = read_hex("subsystem_device", dir);
    auto str = [dir](const char* name) {
        auto v = read_attr(name, dir);
        return v ? trim(*v) : std::string();
    };
    d.max_link_speed = str("max_link_speed");
    d.max_link_width = read_int("max_link_width", 0, dir);
    // The port above: the parent directory (the path is canonical, so ".." is its dirname).
    d.port_max_link_speed = str("../max_link_speed");
    d.port_max_link_width = read_int("../max_link_width", 0, dir);
}

bool read_topo_attrs(PciDev& d) {
    if (d.topo_attrs) return true;
    const int dir = ::open(d.path.c_str(), O_PATH | O_DIRECTORY | O_CLOEXEC);
    if (dir < 0) return false;
    topo_attrs_at(dir, d);
    ::close(dir);
    return true;
}

std::optional<PciDev> read_pci_dir(const std::string& real, bool topo_attrs, bool with_driver) {
    PciDev d;
    d.path = real;
    d.bdf = path_basename(real);
    if (!looks_like_bdf(d.bdf)) return std::nullopt;
    auto pos = real.find("/devices/");
    if (pos == std::string::npos) return std::nullopt;
    const int dir = ::open(real.c_str(), O_PATH | O_DIRECTORY | O_CLOEXEC);
    if (dir < 0) return std::nullopt;
    struct CloseDir {
        int fd;
        ~CloseDir() { ::close(fd); }
    } guard{dir};
    for (auto& c : split(real.substr(pos + 9), '/'))
        if (!c.empty()) d.chain.push_back(c);
    if (with_driver) {  // "driver" is a symlink to .../drivers/<name>: its last component is all we need
        char buf[PATH_MAX];
        ssize_t n = ::readlinkat(dir, "driver", buf, sizeof buf - 1);
        if (n > 0) d.driver = path_basename(std::string(buf, size_t(n)));
    }
    d.vendor = read_hex("vendor", dir);
    d.device = read_hex("device", dir);
    d.pci_class = read_hex("class", dir);
    d.numa = read_int("numa_node", -1, dir);
    if (topo_attrs) topo_attrs_at(dir, d);
    return d;
}

std::string PciDev::rccl_link_speed() const {
    float dev = FLT_MAX, port = FLT_MAX;
    std::sscanf(max_link_speed.c_str(), "%f GT/s", &dev);
    std::sscanf(port_max_link_speed.c_str(), "%f GT/s", &port);
    return port < dev ? port_max_link_speed : max_link_speed;
}

int PciDev::rccl_link_width() const { return std::min(max_link_width, port_max_link_width); }

CpuIdentity cpu_identity() {
    CpuIdentity c;
    utsname u{};
    if (::uname(&u) == 0) c.arch = u.machine;
#if defined(__x86_64__)
    unsigned a = 0, b = 0, cx = 0, d = 0;
    if (__get_cpuid(0, &a, &b, &cx, &d)) {
        char v[13] = {};
        std::memcpy(v, &b, 4);
        std::memcpy(v + 4, &d, 4);
        std::memcpy(v + 8, &cx, 4);
        c.vendor = v;
    }
    if (__get_cpuid(1, &a, &b, &cx, &d)) {
        unsigned model = (a >> 4) & 0xf, family = (a >> 8) & 0xf, ext_model = (a >> 16) & 0xf, ext_family = (a >> 20) & 0xff;
        c.family = int(family + (ext_family << 4));
        c.model = int(model + (ext_model << 4));
    }
#endif
    return c;
}

std::string numa_cpumap(const std::string& root, int numa) {
    if (numa < 0) return "";
    auto s = read_file(path_join(root, "devices/system/node/node" + std::to_string(numa) + "/cpumap"));
    return s ? trim(*s) : "";
}

std::optional<PciDev> netdev_pci(const std::string& root, const std::string& ifname) {
    if (ifname.empty() || ifname.find('/') != std::string::npos) return std::nullopt;
    return read_pci_dev(root, path_join(root, "class/net/" + ifname + "/device"));
}

int64_t netdev_speed_mbps(const std::string& root, const std::string& ifname) {
    if (ifname.empty() || ifname.find('/') != std::string::npos) return -1;
    auto s = read_file(path_join(root, "class/net/" + ifname + "/speed"));
    if (!s) return -1;
    try {
        const long long v = std::stoll(trim(*s));
        return v > 0 ? int64_t(v) : -1;  // the kernel reports -1 (SPEED_UNKNOWN) while down
    } catch (const std::exception&) {
        return -1;
    }
}

std::string netdev_rdma_device(const std::string& root, const std::string& ifname) {
    if (ifname.empty() || ifname.find('/') != std::string::npos) return "";
    auto ib = list_dir(path_join(root, "class/net/" + ifname + "/device/infiniband"));
    return ib.empty() ? std::string() : ib.front();
}

std::vector<std::string> netdev_uppers(const std::string& root, const std::string& ifname) {
    std::vector<std::string> out;
    if (ifname.empty() || ifname.find('/') != std::string::npos) return out;
    for (auto& e : list_dir(path_join(root, "class/net/" + ifname)))
        if (e.rfind("upper_", 0) == 0 && e.size() > 6) out.push_back(e.substr(6));
    std::sort(out.begin(), out.end());
    return out;
}

std::vector<PciDev> rccl_pci_parents(const PciDev& d, std::map<std::string, PciDev>* cache) {
    std::vector<PciDev> out;
    auto pos = d.path.find("/devices/");
    if (pos == std::string::npos || d.chain.empty()) return out;
    const std::string prefix = d.path.substr(0, pos + 8);  // ".../devices"
    auto dir_of = [&](size_t k) {
        std::string p = prefix;
        for (size_t i = 0; i <= k; ++i) p += "/" + d.chain[i];
        return p;
    };
    size_t i = d.chain.size() - 1;
    while (i >= 2 && looks_like_bdf(d.chain[i - 1]) && looks_like_bdf(d.chain[i - 2])) {
        i -= 2;
        const std::string dir = dir_of(i);
        if (cache) {
            auto it = cache->find(dir);
            if (it != cache->end()) {
                out.push_back(it->second);
                continue;
            }
        }
        auto p = read_pci_dir(dir, true, false);  // a bridge's driver (pcieport) is not needed
        if (!p) break;  // unreadable bridge: RCCL would stop there too (no sysfs entry)
        if (cache) cache->emplace(dir, *p);
        out.push_back(std::move(*p));
    }
    std::reverse(out.begin(), out.end());
    return out;
}

std::vector<Gpu> discover_gpus(const std::string& root, const std::string& driver) {
    std::vector<Gpu> out;
    std::string dir = path_join(root, "bus/pci/drivers/" + driver);
    for (auto& name : list_dir(dir)) {
        if (!looks_like_bdf(name)) continue;
        auto d = read_pci_dev(root, path_join(dir, name), false);
        if (!d) {
            NLOG_W("Expected '%s' to be a symlink to a PCI device", path_join(dir, name).c_str());
            continue;
        }
        if (d->driver.empty()) d->driver = driver;
        Gpu g;
        g.pci = *d;
        out.push_back(std::move(g));
    }
    std::sort(out.begin(), out.end(), [](const Gpu& a, const Gpu& b) { return a.pci.bdf < b.pci.bdf; });
    for (size_t i = 0; i < out.size(); ++i) out[i].index = int(i);
    return out;
}

std::vector<Nic> discover_pci_nics(const std::string& root, const std::vector<std::string>& drivers) {
    std::vector<Nic> out;
    std::string cls = path_join(root, "class/net");
    for (auto& ifname : list_dir(cls)) {
        auto real = realpath_of(path_join(cls, ifname));
        if (!real) continue;
        // <pci device dir>/net/<ifname>
        std::string netdir = path_dirname(*real);
        if (path_basename(netdir) != "net") continue;
        std::string devdir = path_dirname(netdir);
        if (!looks_like_bdf(path_basename(devdir))) continue;  // virtual / non-PCI netdev
        auto d = read_pci_dev(root, devdir, false);
        if (!d) continue;
        if (!drivers.empty() && std::find(drivers.begin(), drivers.end(), d->driver) == drivers.end()) continue;
        Nic n;
        n.ifname = ifname;
        n.pci = *d;
        if (auto a = read_file(path_join(*real, "address")))
            if (auto m = MacAddr::parse(trim(*a))) n.mac = *m;
        auto ib = list_dir(path_join(devdir, "infiniband"));
        if (!ib.empty()) n.rdma_dev = ib.front();
        n.rdma_port = read_int(path_join(*real, "dev_port"), 0) + 1;
        out.push_back(std::move(n));
    }
    std::sort(out.begin(), out.end(), [](const Nic& a, const Nic& b) {
        return a.pci.bdf != b.pci.bdf ? a.pci.bdf < b.pci.bdf : a.ifname < b.ifname;
    });
    return out;
}

PathType path_between(const PciDev& a, const PciDev& b, int* common_depth) {
    size_t n = 0;
    while (n < a.chain.size() && n < b.chain.size() && a.chain[n] == b.chain[n]) ++n;
    if (common_depth) *common_depth = int(n);
    // chain[0] = host bridge "pciDDDD:BB", chain[1] = root port, chain[2..] = switch ports.
    // Sharing a component past the root port means both sit below one PCIe switch.
    if (n >= 3) {
        // Diverging right below one switch's upstream port ([downstream port, endpoint] left on
        // each side) is a single bridge (PIX); anything deeper crosses several switches (PXB).
        size_t da = a.chain.size() - n, db = b.chain.size() - n;
        return (da <= 2 && db <= 2) ? PathType::PIX : PathType::PXB;
    }
    if (n >= 1) return PathType::PHB;
    if (a.numa >= 0 && a.numa == b.numa) return PathType::NODE;
    return PathType::SYS;
}

std::vector<GpuNicPair> pair_gpus_nics(const std::vector<Gpu>& gpus, const std::vector<Nic>& nics, PathType max_path) {
    std::vector<GpuNicPair> out;
    std::vector<bool> used(nics.size(), false);
    for (size_t g = 0; g < gpus.size(); ++g) {
        int best = -1, best_depth = -1;
        PathType best_path = PathType::SYS;
        for (size_t n = 0; n < nics.size(); ++n) {
            if (used[n]) continue;
            int depth = 0;
            PathType p = path_between(gpus[g].pci, nics[n].pci, &depth);
            if (int(p) > int(max_path)) continue;
            if (best < 0 || int(p) < int(best_path) || (p == best_path && depth > best_depth)) {
                best = int(n);
                best_depth = depth;
                best_path = p;
            }
        }
        if (best >= 0) {
            used[size_t(best)] = true;
            out.push_back(GpuNicPair{int(g), best, best_path, best_depth});
        }
    }
    return out;
}

std::vector<std::string> accel_netdevs(const std::string& root, const std::string& driver) {
    std::vector<std::string> out;
    std::string dir = path_join(root, "bus/pci/drivers/" + driver);
    for (auto& name : list_dir(dir)) {
        if (!looks_like_bdf(name)) continue;
        auto real = realpath_of(path_join(dir, name));
        if (!real) {
            NLOG_W("Expected '%s' to be a symlink", path_join(dir, name).c_str());
            continue;
        }
        for (auto& n : list_dir(path_join(*real, "net"))) out.push_back(n);
    }
    return out;
}

DiscoveryResult discover(const DiscoveryOptions& opt, const std::string& root) {
    DiscoveryResult r;
    if (opt.mode == DiscoveryMode::None) return r;
    if (opt.mode == DiscoveryMode::Accel) {
        r.ifnames = accel_netdevs(root, opt.accel_driver);
        return r;
    }
    if (opt.mode == DiscoveryMode::Rdma) {
        // The accelerators are enumerated only to know which NICs are theirs.
        const std::vector<Gpu> gpus = opt.exclude_gpu_rails ? discover_gpus(root, opt.accel_driver) : std::vector<Gpu>{};
        for (auto& n : discover_pci_nics(root, opt.nic_drivers)) {
            if (n.rdma_dev.empty()) continue;
            const Gpu* rail_of = nullptr;
            PathType path = PathType::SYS;
            for (const auto& g : gpus) {
                PathType p = path_between(g.pci, n.pci);
                if (int(p) <= int(opt.gpu_rail_path) && (!rail_of || int(p) < int(path))) {
                    rail_of = &g;
                    path = p;
                }
            }
            if (rail_of) {
                r.excluded.emplace_back(n.ifname, strfmt("scale-out rail of GPU %s (%s, path %s): the amd-so agent's NIC",
                                                         rail_of->pci.bdf.c_str(), opt.accel_driver.c_str(),
                                                         to_string(path)));
                continue;
            }
            r.ifnames.push_back(n.ifname);
            r.nics.push_back(std::move(n));
        }
        return r;
    }
    r.gpus = discover_gpus(root, opt.accel_driver);
    r.nics = discover_pci_nics(root, opt.nic_drivers);
    r.pairs = pair_gpus_nics(r.gpus, r.nics, opt.max_path);
    for (auto& p : r.pairs) r.ifnames.push_back(r.nics[size_t(p.nic)].ifname);
    return r;
}

static std::optional<std::array<uint8_t, 16>> parse_gid(const std::string& s) {
    // "0000:0000:0000:0000:0000:ffff:0a00:0001"
    auto parts = split(trim(s), ':');
    if (parts.size() != 8) return std::nullopt;
    std::array<uint8_t, 16> g{};
    for (size_t i = 0; i < 8; ++i) {
        if (parts[i].empty() || parts[i].size() > 4) return std::nullopt;
        char* end = nullptr;
        unsigned long v = std::strtoul(parts[i].c_str(), &end, 16);
        if (*end) return std::nullopt;
        g[i * 2] = uint8_t(v >> 8);
        g[i * 2 + 1] = uint8_t(v);
    }
    return g;
}

std::optional<int> find_rocev2_linklocal_gid_index(const std::string& root, const std::string& rdma_dev, int port) {
    std::string pdir = path_join(root, "class/infiniband/" + rdma_dev + "/ports/" + std::to_string(port));
    std::vector<int> idx;
    for (auto& n : list_dir(path_join(pdir, "gids"))) {
        char* end = nullptr;
        long v = std::strtol(n.c_str(), &end, 10);
        if (*end == 0) idx.push_back(int(v));
    }
    std::sort(idx.begin(), idx.end());
    for (int i : idx) {
        auto g = read_attr(path_join(pdir, "gids/" + std::to_string(i)));
        if (!g) continue;
        auto gid = parse_gid(*g);
        if (!gid || (*gid)[0] != 0xfe || ((*gid)[1] & 0xc0) != 0x80) continue;  // fe80::/10
        auto type = read_attr(path_join(pdir, "gid_attrs/types/" + std::to_string(i)));
        if (type && trim(*type) == "RoCE v2") return i;
    }
    return std::nullopt;
}

std::optional<int> find_rocev2_gid_index(const std::string& root, const std::string& rdma_dev, int port, Ipv4 ip) {
    std::string pdir = path_join(root, "class/infiniband/" + rdma_dev + "/ports/" + std::to_string(port));
    auto names = list_dir(path_join(pdir, "gids"));
    std::vector<int> idx;
    for (auto& n : names) {
        char* end = nullptr;
        long v = std::strtol(n.c_str(), &end, 10);
        if (*end == 0) idx.push_back(int(v));
    }
    std::sort(idx.begin(), idx.end());
    std::array<uint8_t, 16> want{};
    want[10] = want[11] = 0xff;
    ip.to_net(&want[12]);
    for (int i : idx) {
        auto g = read_attr(path_join(pdir, "gids/" + std::to_string(i)));
        if (!g) continue;
        auto gid = parse_gid(*g);
        if (!gid || *gid != want) continue;
        auto type = read_attr(path_join(pdir, "gid_attrs/types/" + std::to_string(i)));
        if (type && trim(*type) == "RoCE v2") return i;
    }
    return std::nullopt;
}

// ---------------------------------------------------------------------------
// KFD topology
// ---------------------------------------------------------------------------
static std::map<std::string, std::string> read_props(const std::string& path) {
    std::map<std::string, std::string> m;
    auto s = read_file(path);
    if (!s) return m;
    for (auto& line : split(*s, '\n')) {
        auto f = split_ws(line);
        if (f.size() >= 2) m[f[0]] = f[1];
    }
    return m;
}

static uint64_t prop_u64(const std::map<std::string, std::string>& m, const char* k) {
    auto it = m.find(k);
    return it == m.end() ? 0 : std::strtoull(it->second.c_str(), nullptr, 10);
}

std::string KfdNode::bdf() const {
    return strfmt("%04x:%02x:%02x.%x", domain, (location_id >> 8) & 0xff, (location_id >> 3) & 0x1f, location_id & 7);
}

uint64_t XgmiReport::per_gpu_bw_mbs() const {
    if (gpus.empty()) return 0;
    uint64_t best = UINT64_MAX;
    for (auto& g : gpus) {
        uint64_t sum = 0;
        std::set<int> peers;
        for (auto& l : links) {
            int peer = l.from == g.node ? l.to : (l.to == g.node ? l.from : -1);
            if (peer < 0 || !peers.insert(peer).second) continue;
            sum += l.max_bw_mbs;
        }
        best = std::min(best, sum);
    }
    return best == UINT64_MAX ? 0 : best;
}

XgmiReport read_xgmi(const std::string& root) {
    XgmiReport r;
    std::string base = path_join(root, "class/kfd/kfd/topology/nodes");
    std::map<int, KfdNode> nodes;
    std::vector<KfdLink> all;
    for (auto& n : list_dir(base)) {
        char* end = nullptr;
        long id = std::strtol(n.c_str(), &end, 10);
        if (*end) continue;
        auto props = read_props(path_join(base, n + "/properties"));
        KfdNode k;
        k.node = int(id);
        k.simd_count = uint32_t(prop_u64(props, "simd_count"));
        k.vendor_id = uint32_t(prop_u64(props, "vendor_id"));
        k.device_id = uint32_t(prop_u64(props, "device_id"));
        k.location_id = uint32_t(prop_u64(props, "location_id"));
        k.domain = uint32_t(prop_u64(props, "domain"));
        k.hive_id = prop_u64(props, "hive_id");
        k.num_xcc = uint32_t(prop_u64(props, "num_xcc"));
        if (auto g = read_file(path_join(base, n + "/gpu_id"))) k.gpu_id = uint32_t(std::strtoul(trim(*g).c_str(), nullptr, 10));
        nodes[k.node] = k;
        for (const char* sub : {"io_links", "p2p_links"}) {
            std::string ldir = path_join(base, n + "/" + sub);
            for (auto& l : list_dir(ldir)) {
                auto lp = read_props(path_join(ldir, l + "/properties"));
                if (lp.empty()) continue;  // unreadable (e.g. filtered in a container)
                KfdLink link;
                link.type = int(prop_u64(lp, "type"));
                link.from = int(prop_u64(lp, "node_from"));
                link.to = int(prop_u64(lp, "node_to"));
                link.weight = int(prop_u64(lp, "weight"));
                link.min_bw_mbs = uint32_t(prop_u64(lp, "min_bandwidth"));
                link.max_bw_mbs = uint32_t(prop_u64(lp, "max_bandwidth"));
                all.push_back(link);
            }
        }
    }
    // A GPU node whose properties were filtered reads simd_count 0; a node that is the
    // endpoint of an xGMI link is a GPU regardless.
    std::set<int> xgmi_nodes;
    for (auto& l : all)
        if (l.type == kIoLinkTypeXgmi) {
            xgmi_nodes.insert(l.from);
            xgmi_nodes.insert(l.to);
        }
    for (auto& [id, k] : nodes)
        if (k.is_gpu() || xgmi_nodes.count(id)) r.gpus.push_back(k);
    std::sort(r.gpus.begin(), r.gpus.end(), [](const KfdNode& a, const KfdNode& b) {
        return a.is_gpu() != b.is_gpu() ? a.is_gpu() : (a.location_id != b.location_id ? a.location_id < b.location_id : a.node < b.node);
    });

    std::set<std::pair<int, int>> connected;
    uint64_t minbw = UINT64_MAX;
    for (auto& l : all) {
        if (l.type != kIoLinkTypeXgmi) continue;
        r.links.push_back(l);
        connected.insert({std::min(l.from, l.to), std::max(l.from, l.to)});
        if (l.max_bw_mbs) minbw = std::min<uint64_t>(minbw, l.max_bw_mbs);
    }
    r.min_link_bw_mbs = minbw == UINT64_MAX ? 0 : minbw;
    int n = int(r.gpus.size());
    r.pairs_expected = n * (n - 1) / 2;
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) {
            int a = std::min(r.gpus[size_t(i)].node, r.gpus[size_t(j)].node);
            int b = std::max(r.gpus[size_t(i)].node, r.gpus[size_t(j)].node);
            if (connected.count({a, b}))
                ++r.pairs_connected;
            else
                r.missing.emplace_back(r.gpus[size_t(i)].bdf(), r.gpus[size_t(j)].bdf());
        }
    return r;
}

// ---------------------------------------------------------------------------
// PCIe link state
// ---------------------------------------------------------------------------
std::string PcieLink::str() const {
    if (!known()) return "unknown";
    std::string s = strfmt("%.1f GT/s x%d", speed_gts, width);
    if (degraded()) s += strfmt(" of %.1f GT/s x%d", max_speed_gts, max_width);
    return s;
}

PcieLink read_pcie_link(const std::string& root, const std::string& bdf) {
    PcieLink l;
    const std::string dir = path_join(root, "bus/pci/devices/" + bdf);
    auto gts = [&](const char* attr) {  // "32.0 GT/s PCIe"; "Unknown" (a link that is down) reads 0
        auto v = read_attr(path_join(dir, attr));
        return v ? std::strtod(v->c_str(), nullptr) : 0.0;
    };
    auto lanes = [&](const char* attr) {
        auto v = read_attr(path_join(dir, attr));
        return v ? int(std::strtol(v->c_str(), nullptr, 10)) : 0;
    };
    l.speed_gts = gts("current_link_speed");
    l.max_speed_gts = gts("max_link_speed");
    l.width = lanes("current_link_width");
    l.max_width = lanes("max_link_width");
    // The link can train no faster or wider than the port above it supports (a Gen5 card in a
    // Gen4 slot is not degraded): the maximum is the lower of the two ends'.
    char real[PATH_MAX];
    if (::realpath(dir.c_str(), real)) {
        const std::string up = path_dirname(real);
        auto v = read_attr(path_join(up, "max_link_speed"));
        const double up_gts = v ? std::strtod(v->c_str(), nullptr) : 0.0;
        auto w = read_attr(path_join(up, "max_link_width"));
        const int up_width = w ? int(std::strtol(w->c_str(), nullptr, 10)) : 0;
        if (up_gts > 0) l.max_speed_gts = std::min(l.max_speed_gts, up_gts);
        if (up_width > 0) l.max_width = std::min(l.max_width, up_width);
    }
    return l;
}

// ---------------------------------------------------------------------------
// xGMI link health (gpu_metrics)
// ---------------------------------------------------------------------------
namespace {
// gpu_metrics 1.8: a 4-byte header (u16 structure_size, u8 format_revision, u8 content_revision),
// then the fields; the xGMI ones sit at these offsets (little-endian, as the GPU writes them).
constexpr size_t kGm18Width = 72, kGm18Speed = 74, kGm18Read = 136, kGm18Write = 200, kGm18Status = 264;
constexpr size_t kGm18End = kGm18Status + 2 * kMaxXgmiLinks;

template <typename T>
T le_at(const std::string& b, size_t off) {
    T v{};
    std::memcpy(&v, b.data() + off, sizeof v);
    return v;
}
}  // namespace

int XgmiLinkHealth::links_up() const { return int(std::count(status.begin(), status.end(), 1)); }
int XgmiLinkHealth::links_down() const { return int(std::count(status.begin(), status.end(), 0)); }

XgmiLinkHealth parse_gpu_metrics(const std::string& blob) {
    XgmiLinkHealth h;
    if (blob.size() < 4) {
        h.error = "gpu_metrics unreadable or empty";
        return h;
    }
    const int format = uint8_t(blob[2]), content = uint8_t(blob[3]);
    h.revision = strfmt("%d.%d", format, content);
    if (format != 1 || content != 8) {
        h.error = "gpu_metrics " + h.revision + " is not a layout this agent reads (1.8): xGMI link state not checked";
        return h;
    }
    if (blob.size() < kGm18End || le_at<uint16_t>(blob, 0) < kGm18End) {
        h.error = strfmt("gpu_metrics 1.8 truncated (%zu bytes)", blob.size());
        return h;
    }
    h.known = true;
    h.width = le_at<uint16_t>(blob, kGm18Width);
    h.speed_gbps = le_at<uint16_t>(blob, kGm18Speed);
    for (int i = 0; i < kMaxXgmiLinks; ++i) {
        const uint16_t st = le_at<uint16_t>(blob, kGm18Status + 2 * size_t(i));
        h.status.push_back(st == 1 ? 1 : st == 0 ? 0 : -1);  // 0xffff: no link in this slot
        h.read_kb.push_back(le_at<uint64_t>(blob, kGm18Read + 8 * size_t(i)));
        h.write_kb.push_back(le_at<uint64_t>(blob, kGm18Write + 8 * size_t(i)));
    }
    return h;
}

std::vector<XgmiLinkHealth> read_xgmi_health(const std::string& root, const std::vector<std::string>& bdfs) {
    std::vector<XgmiLinkHealth> out;
    for (const auto& bdf : bdfs) {
        auto blob = read_file(path_join(root, "bus/pci/devices/" + bdf + "/gpu_metrics"));
        XgmiLinkHealth h = parse_gpu_metrics(blob ? *blob : std::string());
        h.bdf = bdf;
        out.push_back(std::move(h));
    }
    return out;
}

std::vector<XgmiLinkHealth> read_xgmi_health(const std::string& root, const std::vector<std::string>& bdfs,
                                             int64_t timeout_ns) {
    std::vector<std::string> paths;
    for (const auto& bdf : bdfs) paths.push_back(path_join(root, "bus/pci/devices/" + bdf + "/gpu_metrics"));
    const auto reads = bounded::read_files(paths, mono_ns() + timeout_ns);
    std::vector<XgmiLinkHealth> out;
    for (size_t i = 0; i < bdfs.size(); ++i) {
        XgmiLinkHealth h;
        if (reads[i].late) {
            h.late = true;
            h.error = "gpu_metrics did not answer in " + format_go_duration(timeout_ns);
        } else {
            h = parse_gpu_metrics(reads[i].data ? *reads[i].data : std::string());
        }
        h.bdf = bdfs[i];
        out.push_back(std::move(h));
    }
    return out;
}

// ---------------------------------------------------------------------------
// GPUDirect RDMA
// ---------------------------------------------------------------------------
bool kernel_at_least(const std::string& release, int major, int minor) {
    int ma = 0, mi = 0;
    if (std::sscanf(release.c_str(), "%d.%d", &ma, &mi) != 2) return false;
    return ma > major || (ma == major && mi >= minor);
}

GdrReport detect_gdr(const std::string& root, const std::string& kernel_release) {
    GdrReport g;
    if (auto v = read_file(path_join(root, "kernel/mm/memory_peers/amdkfd/version"))) {
        g.peer_mem = true;
        g.peer_mem_version = trim(*v);
    }
    g.ib_uverbs = path_exists(path_join(root, "module/ib_uverbs"));
    g.kernel = kernel_release;
    if (g.kernel.empty()) {
        utsname u{};
        if (::uname(&u) == 0) g.kernel = u.release;
    }
    g.dmabuf = g.ib_uverbs && kernel_at_least(g.kernel, 5, 12);
    return g;
}

}  // namespace netop::topo
