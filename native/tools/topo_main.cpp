// `netop-topo` — prints the node's scale-out topology as JSON: amdgpu GPUs, candidate
// NICs, GPU<->NIC pairing (PCIe path type), RDMA devices, the xGMI mesh from KFD, and which
// RDMA NICs a host-nic policy's discovery would take (the GPU rails left to amd-so).
// Used by the readiness tooling, the GPU-box smoke test and fake-sysfs tests.
#include <cstdio>

#include "netop/artifacts.hpp"
#include "netop/cli.hpp"
#include "netop/topology.hpp"

using namespace netop;

int main(int argc, char** argv) {
    std::string root, nic_drivers;
    bool all_drivers = false;
    cli::FlagSet fs("netop-topo");
    fs.add_string("sysfs-root", &root, "sysfs root (default $SYSFS_ROOT or /sys/)");
    fs.add_string("nic-drivers", &nic_drivers, "comma separated NIC driver allow-list");
    fs.add_bool("all-drivers", &all_drivers, "consider every PCI network driver");
    try {
        fs.parse(argc, argv);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error: %s\n", e.what());
        return 2;
    }
    if (root.empty()) root = topo::sysfs_root();
    topo::DiscoveryOptions opt;
    if (!nic_drivers.empty()) opt.nic_drivers = split(nic_drivers, ',');
    if (all_drivers) opt.nic_drivers.clear();
    auto d = topo::discover(opt, root);
    auto x = topo::read_xgmi(root);
    std::vector<std::string> bdfs;
    for (auto& g : d.gpus) bdfs.push_back(g.pci.bdf);
    auto health = topo::read_xgmi_health(root, bdfs);

    artifacts::Json j;
    auto pcie = [&](const std::string& bdf) {
        auto l = topo::read_pcie_link(root, bdf);
        j.begin_object().key("known").value(l.known()).key("degraded").value(l.degraded()).key("str").value(l.str());
        j.end_object();
    };
    j.begin_object();
    j.key("gpus").begin_array();
    for (size_t i = 0; i < d.gpus.size(); ++i) {
        const auto& g = d.gpus[i];
        j.begin_object().key("index").value(g.index).key("bdf").value(g.pci.bdf).key("device").value(strfmt("0x%04x", g.pci.device));
        j.key("numa").value(g.pci.numa).key("driver").value(g.pci.driver);
        j.key("pcie");
        pcie(g.pci.bdf);
        const auto& h = health[i];  // xGMI links as trained: "U" up, "D" down, "X" no link in the slot
        j.key("xgmi_links").begin_object().key("known").value(h.known);
        if (h.known) {
            std::string st;
            for (int v : h.status) st += v == 1 ? 'U' : v == 0 ? 'D' : 'X';
            j.key("revision").value(h.revision).key("status").value(st).key("up").value(h.links_up());
            j.key("down").value(h.links_down()).key("width").value(h.width).key("speed_gbps").value(h.speed_gbps);
        } else {
            j.key("error").value(h.error);
        }
        j.end_object().end_object();
    }
    j.end_array();
    j.key("nics").begin_array();
    for (auto& n : d.nics) {
        j.begin_object().key("ifname").value(n.ifname).key("bdf").value(n.pci.bdf).key("driver").value(n.pci.driver);
        j.key("numa").value(n.pci.numa).key("rdma_dev").value(n.rdma_dev).key("mac").value(n.mac.str()).key("pcie");
        pcie(n.pci.bdf);
        j.end_object();
    }
    j.end_array();
    j.key("pairs").begin_array();
    for (auto& p : d.pairs) {
        j.begin_object().key("gpu").value(d.gpus[size_t(p.gpu)].pci.bdf).key("nic").value(d.nics[size_t(p.nic)].ifname);
        j.key("path").value(topo::to_string(p.path)).key("common_depth").value(p.common_depth).end_object();
    }
    j.end_array();
    {
        // What host-nic (rdma) discovery takes from sysfs alone; the agent then also leaves out
        // the node's own NICs, which needs rtnetlink (default route, addresses, routes, bonds).
        topo::DiscoveryOptions ro = opt;
        ro.mode = topo::DiscoveryMode::Rdma;
        auto r = topo::discover(ro, root);
        j.key("host_nics").begin_object().key("ifnames").begin_array();
        for (const auto& n : r.ifnames) j.value(n);
        j.end_array().key("left_alone").begin_object();
        for (const auto& [n, why] : r.excluded) j.key(n).value(why);
        j.end_object().end_object();
    }
    j.key("xgmi").begin_object();
    j.key("gpus").begin_array();
    for (auto& g : x.gpus) j.value(g.bdf());
    j.end_array();
    j.key("links").value(int64_t(x.links.size()));
    j.key("pairs_expected").value(x.pairs_expected).key("pairs_connected").value(x.pairs_connected);
    j.key("full_mesh").value(x.full_mesh());
    j.key("min_link_bw_mbs").value(x.min_link_bw_mbs).key("per_gpu_bw_mbs").value(x.per_gpu_bw_mbs());
    j.end_object();
    j.end_object();
    std::printf("%s\n", j.str().c_str());
    return 0;
}
