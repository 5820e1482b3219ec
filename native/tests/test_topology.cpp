#include "check.hpp"
#include "netop/topology.hpp"
#include "tmpdir.hpp"

using namespace netop;
using namespace netop::topo;

namespace {
// Builds a fake sysfs PCI device directory with a driver symlink.
void pci(const TmpDir& t, const std::string& path, const char* driver, const char* vendor, const char* device, int numa) {
    t.mkdir("devices/" + path);
    t.write("devices/" + path + "/vendor", std::string(vendor) + "\n");
    t.write("devices/" + path + "/device", std::string(device) + "\n");
    t.write("devices/" + path + "/numa_node", std::to_string(numa) + "\n");
    t.mkdir(std::string("bus/pci/drivers/") + driver);
    t.symlink(std::string("bus/pci/drivers/") + driver, "devices/" + path + "/driver");
}
void netdev(const TmpDir& t, const std::string& pcipath, const std::string& ifname, const char* mac) {
    t.write("devices/" + pcipath + "/net/" + ifname + "/address", std::string(mac) + "\n");
    t.symlink("devices/" + pcipath + "/net/" + ifname, "class/net/" + ifname);
}
void build_node(const TmpDir& t) {
    // Two GPUs, each behind a switch with a NIC (same layout as a real MI355X node), plus a
    // management NIC on its own root port and a virtual interface.
    const std::string g0 = "pci0000:00/0000:00:01.1/0000:01:00.0/0000:02:08.0/0000:06:00.0/0000:07:10.0/0000:08:00.0/0000:09:00.0/0000:0a:00.0";
    const std::string n0 = "pci0000:00/0000:00:01.1/0000:01:00.0/0000:02:00.0/0000:03:00.0/0000:04:10.0/0000:05:00.0";
    const std::string g1 = "pci0000:19/0000:19:01.1/0000:1a:00.0/0000:1b:08.0/0000:1f:00.0/0000:20:10.0/0000:21:00.0/0000:22:00.0/0000:23:00.0";
    const std::string n1 = "pci0000:19/0000:19:01.1/0000:1a:00.0/0000:1b:00.0/0000:1c:00.0/0000:1d:10.0/0000:1e:00.0";
    const std::string mg = "pci0000:37/0000:37:01.1/0000:38:00.0";
    pci(t, g0, "amdgpu", "0x1002", "0x75a3", 0);
    pci(t, g1, "amdgpu", "0x1002", "0x75a3", 0);
    pci(t, n0, "mlx5_core", "0x15b3", "0x1021", 0);
    pci(t, n1, "mlx5_core", "0x15b3", "0x1021", 0);
    pci(t, mg, "mlx5_core", "0x15b3", "0x1021", 0);
    t.symlink("devices/" + g0, "bus/pci/drivers/amdgpu/0000:0a:00.0");
    t.symlink("devices/" + g1, "bus/pci/drivers/amdgpu/0000:23:00.0");
    netdev(t, n0, "enp5s0np0", "02:00:00:00:00:05");
    netdev(t, n1, "enp30s0np0", "02:00:00:00:00:30");
    netdev(t, mg, "ens9np0", "02:00:00:00:00:09");
    t.mkdir("devices/" + n1 + "/infiniband/mlx5_3");
    t.mkdir("devices/" + n0 + "/infiniband/mlx5_1");
    t.write("devices/virtual/net/lo/address", "00:00:00:00:00:00\n");
    t.symlink("devices/virtual/net/lo", "class/net/lo");
}
}  // namespace

TEST(topology_affine_pairing_excludes_mgmt_nic) {
    TmpDir t;
    build_node(t);
    DiscoveryOptions opt;
    auto r = discover(opt, t.path);
    CHECK_EQ(r.gpus.size(), size_t(2));
    CHECK_EQ(r.gpus[0].pci.bdf, std::string("0000:0a:00.0"));
    CHECK_EQ(r.gpus[0].pci.device, uint32_t(0x75a3));
    CHECK_EQ(r.nics.size(), size_t(3));
    CHECK_EQ(r.pairs.size(), size_t(2));
    CHECK_EQ(r.ifnames.size(), size_t(2));
    CHECK_EQ(r.ifnames[0], std::string("enp5s0np0"));
    CHECK_EQ(r.ifnames[1], std::string("enp30s0np0"));
    CHECK_EQ(r.nics[size_t(r.pairs[1].nic)].rdma_dev, std::string("mlx5_3"));
    CHECK(r.pairs[0].path == PathType::PXB);
    CHECK_EQ(r.pairs[0].common_depth, 3);
    // Accepting anything up to SYS would still pair each GPU with its own switch-local NIC.
    opt.max_path = PathType::SYS;
    auto r2 = discover(opt, t.path);
    CHECK_EQ(r2.ifnames[0], std::string("enp5s0np0"));
    // Driver allow-list filters NICs.
    opt.nic_drivers = {"bnxt_en"};
    CHECK(discover(opt, t.path).ifnames.empty());
}

TEST(topology_accel_mode_reference_compatible) {
    TmpDir t;
    // habanalabs-style: netdevs directly under the accelerator PCI function.
    const std::string d = "pci0000:00/0000:00:02.0/0000:33:00.0";
    pci(t, d, "habanalabs", "0x1da3", "0x1020", 0);
    t.symlink("devices/" + d, "bus/pci/drivers/habanalabs/0000:33:00.0");
    t.write("devices/" + d + "/net/eth_a/address", "02:00:00:00:00:01\n");
    t.write("devices/" + d + "/net/eth_b/address", "02:00:00:00:00:02\n");
    DiscoveryOptions opt;
    opt.mode = DiscoveryMode::Accel;
    opt.accel_driver = "habanalabs";
    auto r = discover(opt, t.path);
    CHECK_EQ(r.ifnames.size(), size_t(2));
    CHECK(discover(opt, t.path + "/nonexistent").ifnames.empty());
}

TEST(topology_path_types) {
    PciDev a, b;
    a.chain = {"pci0000:00", "0000:00:01.1", "0000:01:00.0", "0000:02:00.0", "0000:03:00.0"};
    b.chain = {"pci0000:00", "0000:00:01.1", "0000:01:00.0", "0000:02:04.0", "0000:04:00.0"};
    CHECK(path_between(a, b) == PathType::PIX);
    b.chain = {"pci0000:00", "0000:00:03.1", "0000:05:00.0"};
    CHECK(path_between(a, b) == PathType::PHB);
    b.chain = {"pci0000:40", "0000:40:01.1", "0000:41:00.0"};
    a.numa = b.numa = 1;
    CHECK(path_between(a, b) == PathType::NODE);
    b.numa = 0;
    CHECK(path_between(a, b) == PathType::SYS);
}

TEST(topology_rocev2_gid_lookup) {
    TmpDir t;
    std::string p = "class/infiniband/mlx5_1/ports/1/";
    t.write(p + "gids/0", "fe80:0000:0000:0000:0000:00ff:fe00:0005\n");
    t.write(p + "gid_attrs/types/0", "IB/RoCE v1\n");
    t.write(p + "gids/1", "fe80:0000:0000:0000:0000:00ff:fe00:0005\n");
    t.write(p + "gid_attrs/types/1", "RoCE v2\n");
    t.write(p + "gids/2", "0000:0000:0000:0000:0000:ffff:0ac8:0001\n");
    t.write(p + "gid_attrs/types/2", "IB/RoCE v1\n");
    t.write(p + "gids/3", "0000:0000:0000:0000:0000:ffff:0ac8:0001\n");
    t.write(p + "gid_attrs/types/3", "RoCE v2\n");
    auto idx = find_rocev2_gid_index(t.path, "mlx5_1", 1, *Ipv4::parse("10.200.0.1"));
    CHECK(idx);
    CHECK_EQ(*idx, 3);
    CHECK(!find_rocev2_gid_index(t.path, "mlx5_1", 1, *Ipv4::parse("10.200.0.5")));
    CHECK(!find_rocev2_gid_index(t.path, "mlx5_9", 1, *Ipv4::parse("10.200.0.1")));
}

TEST(topology_kfd_xgmi_mesh) {
    TmpDir t;
    std::string base = "class/kfd/kfd/topology/nodes/";
    t.write(base + "0/properties", "cpu_cores_count 96\nsimd_count 0\n");
    int n = 4;
    for (int g = 1; g <= n; ++g) {
        t.write(base + std::to_string(g) + "/properties",
                strfmt("simd_count 1024\nvendor_id 4098\ndevice_id 30115\nlocation_id %d\ndomain 0\nhive_id 77\n", (g * 0x10) << 8));
        int li = 0;
        t.write(base + std::to_string(g) + "/io_links/" + std::to_string(li++) + "/properties", "type 2\nnode_from " + std::to_string(g) + "\nnode_to 0\nmax_bandwidth 64000\n");
        for (int h = 1; h <= n; ++h) {
            if (h == g || (g == 1 && h == 4) || (g == 4 && h == 1)) continue;  // 1<->4 missing
            t.write(base + std::to_string(g) + "/io_links/" + std::to_string(li++) + "/properties",
                    strfmt("type 11\nnode_from %d\nnode_to %d\nweight 15\nmin_bandwidth 76000\nmax_bandwidth 76000\n", g, h));
        }
    }
    auto x = read_xgmi(t.path);
    CHECK_EQ(x.gpus.size(), size_t(4));
    CHECK_EQ(x.gpus[0].bdf(), std::string("0000:10:00.0"));
    CHECK_EQ(x.pairs_expected, 6);
    CHECK_EQ(x.pairs_connected, 5);
    CHECK(!x.full_mesh());
    CHECK_EQ(x.missing.size(), size_t(1));
    CHECK_EQ(x.missing[0].first, std::string("0000:10:00.0"));
    CHECK_EQ(x.missing[0].second, std::string("0000:40:00.0"));
    CHECK_EQ(x.min_link_bw_mbs, uint64_t(76000));
    CHECK_EQ(x.per_gpu_bw_mbs(), uint64_t(2 * 76000));
}

TEST(topology_gpu_metrics_1_8_xgmi_links_as_amd_smi_reads_them) {
    // Captured on a live MI355X (tools/gpu_metrics_dump.sh); amd-smi read the same GPU as link
    // status XUUUUUUU, width 16, bit rate 38, link 1 read 7405369007 KB / write 7377082767 KB.
    auto blob = read_file(std::string(NETOP_TEST_FIXTURES) + "/gpu_metrics_v1_8.bin");
    CHECK(blob && blob->size() == 3872);
    auto h = parse_gpu_metrics(*blob);
    CHECK(h.known);
    CHECK_EQ(h.revision, std::string("1.8"));
    CHECK_EQ(h.width, 16);
    CHECK_EQ(h.speed_gbps, 38);
    CHECK(h.status == std::vector<int>({-1, 1, 1, 1, 1, 1, 1, 1}));
    CHECK_EQ(h.links_up(), 7);
    CHECK_EQ(h.links_down(), 0);
    CHECK_EQ(h.read_kb[1], uint64_t(7405369007ULL));
    CHECK_EQ(h.write_kb[1], uint64_t(7377082767ULL));
    CHECK_EQ(h.read_kb[0], uint64_t(0));
    // Link 3 down, as the firmware writes it (0), and link 5 trained at x8.
    std::string down = *blob;
    down[264 + 2 * 3] = 0;
    auto d = parse_gpu_metrics(down);
    CHECK(d.known && d.links_down() == 1 && d.links_up() == 6 && d.status[3] == 0);
    // Another revision: not decoded, and said so; truncated and empty blobs likewise.
    std::string other = *blob;
    other[3] = 7;
    auto o = parse_gpu_metrics(other);
    CHECK(!o.known && o.revision == "1.7" && o.error.find("not a layout") != std::string::npos && o.status.empty());
    CHECK(!parse_gpu_metrics(blob->substr(0, 200)).known);
    CHECK(!parse_gpu_metrics("").known);
    // From sysfs, by BDF; a GPU without the file is reported, not skipped.
    TmpDir t;
    t.write("bus/pci/devices/0000:0a:00.0/gpu_metrics", *blob);
    auto all = read_xgmi_health(t.path, {"0000:0a:00.0", "0000:23:00.0"});
    CHECK_EQ(all.size(), size_t(2));
    CHECK(all[0].known && all[0].bdf == "0000:0a:00.0");
    CHECK(!all[1].known && all[1].bdf == "0000:23:00.0");
}

TEST(topology_pcie_link_trained_vs_supported) {
    TmpDir t;
    const std::string d = "bus/pci/devices/0000:08:00.0/";
    t.write(d + "max_link_speed", "32.0 GT/s PCIe\n");
    t.write(d + "max_link_width", "16\n");
    t.write(d + "current_link_speed", "32.0 GT/s PCIe\n");
    t.write(d + "current_link_width", "16\n");
    auto l = read_pcie_link(t.path, "0000:08:00.0");
    CHECK(l.known() && !l.degraded());
    CHECK_EQ(l.str(), std::string("32.0 GT/s x16"));
    t.write(d + "current_link_width", "8\n");
    t.write(d + "current_link_speed", "16.0 GT/s PCIe\n");
    l = read_pcie_link(t.path, "0000:08:00.0");
    CHECK(l.narrower() && l.slower() && l.degraded());
    CHECK_EQ(l.str(), std::string("16.0 GT/s x8 of 32.0 GT/s x16"));
    t.write(d + "current_link_speed", "Unknown\n");  // a link that is down
    CHECK(!read_pcie_link(t.path, "0000:08:00.0").known());
    CHECK(!read_pcie_link(t.path, "0000:09:00.0").known());  // no such function / no attributes
    // A Gen5 x16 card below a Gen4 x8 port trained as far as the port goes: not degraded.
    const std::string up = "devices/pci0000:40/0000:40:01.0", fn = up + "/0000:41:00.0";
    t.write(up + "/max_link_speed", "16.0 GT/s PCIe\n");
    t.write(up + "/max_link_width", "8\n");
    t.write(fn + "/max_link_speed", "32.0 GT/s PCIe\n");
    t.write(fn + "/max_link_width", "16\n");
    t.write(fn + "/current_link_speed", "16.0 GT/s PCIe\n");
    t.write(fn + "/current_link_width", "8\n");
    t.symlink(fn, "bus/pci/devices/0000:41:00.0");
    auto capped = read_pcie_link(t.path, "0000:41:00.0");
    CHECK(capped.known() && !capped.degraded());
    CHECK_EQ(capped.str(), std::string("16.0 GT/s x8"));
    t.write(fn + "/current_link_width", "4\n");  // but below the port's x8: degraded
    CHECK_EQ(read_pcie_link(t.path, "0000:41:00.0").str(), std::string("16.0 GT/s x4 of 16.0 GT/s x8"));
}

TEST(topology_gdr_detection) {
    TmpDir t;
    auto g = topo::detect_gdr(t.path, "6.8.0-45-generic");
    CHECK_EQ(g.mode(), std::string("none"));
    t.mkdir("module/ib_uverbs");
    CHECK_EQ(topo::detect_gdr(t.path, "6.8.0-45-generic").mode(), std::string("dmabuf"));
    CHECK_EQ(topo::detect_gdr(t.path, "5.4.0-150-generic").mode(), std::string("none"));  // no RDMA dma-buf MRs
    t.mkdir("kernel/mm/memory_peers/amdkfd");
    t.write("kernel/mm/memory_peers/amdkfd/version", "1.0\n");
    auto p = topo::detect_gdr(t.path, "5.4.0");
    CHECK_EQ(p.mode(), std::string("peermem"));
    CHECK_EQ(p.peer_mem_version, std::string("1.0"));
    CHECK(topo::kernel_at_least("5.12.0", 5, 12) && !topo::kernel_at_least("5.11.22", 5, 12));
    CHECK(topo::kernel_at_least("10.0", 5, 12) && !topo::kernel_at_least("garbage", 5, 12));
}

TEST(topology_rdma_mode_lists_host_rdma_nics) {
    TmpDir t;
    // Two mlx5 NICs with RDMA devices, one without (plain Ethernet function), one foreign driver.
    auto nic = [&](const char* bdf, const char* ifname, const char* driver, const char* rdma) {
        std::string dev = std::string("pci0000:00/0000:00:01.0/") + bdf;
        pci(t, dev, driver, "0x15b3", "0x1021", 0);
        netdev(t, dev, ifname, "02:00:00:00:01:01");
        if (rdma) t.mkdir("devices/" + dev + "/infiniband/" + rdma);
    };
    nic("0000:01:00.0", "ens1f0np0", "mlx5_core", "mlx5_0");
    nic("0000:01:00.1", "ens1f1np1", "mlx5_core", "mlx5_1");
    nic("0000:02:00.0", "eno1", "mlx5_core", nullptr);
    nic("0000:03:00.0", "eth7", "e1000e", nullptr);
    DiscoveryOptions o;
    o.mode = DiscoveryMode::Rdma;
    auto r = discover(o, t.path);
    CHECK_EQ(r.ifnames.size(), size_t(2));
    CHECK_EQ(r.ifnames[0], std::string("ens1f0np0"));
    CHECK_EQ(r.nics[1].rdma_dev, std::string("mlx5_1"));
    CHECK(r.pairs.empty() && r.gpus.empty());
    CHECK(parse_discovery_mode("rdma") == DiscoveryMode::Rdma);
}

TEST(topology_rccl_parents_fold_like_rccl) {
    // Layout of GPU 0000:f4:00.0 on a live MI355X box, whose RCCL topology dump
    // (NCCL_TOPO_DUMP_FILE) nests it cpu(numa 1) > e8:00.0 > f0:00.0 > f2:00.0 > f4:00.0.
    TmpDir t;
    const std::string g = "pci0000:e7/0000:e7:01.1/0000:e8:00.0/0000:e9:08.0/0000:f0:00.0/0000:f1:10.0/0000:f2:00.0/0000:f3:00.0/0000:f4:00.0";
    const std::string n = "pci0000:e7/0000:e7:01.1/0000:e8:00.0/0000:e9:00.0/0000:ea:00.0/0000:eb:10.0/0000:ec:00.0/0000:ed:01.0/0000:ef:00.0";
    const std::string m = "pci0000:37/0000:37:01.1/0000:38:00.0";  // NIC straight on a root port
    pci(t, g, "amdgpu", "0x1002", "0x75a3", 1);
    pci(t, n, "ionic", "0x1dd8", "0x1002", 1);
    pci(t, m, "mlx5_core", "0x15b3", "0x1021", 0);
    for (const char* b : {"0000:e8:00.0", "0000:e8:00.0/0000:e9:08.0/0000:f0:00.0"})
        t.write("devices/pci0000:e7/0000:e7:01.1/" + std::string(b) + "/class", "0x060400\n");
    auto gd = read_pci_dev(t.path, t.path + "/devices/" + g);
    CHECK(gd.has_value());
    auto p = rccl_pci_parents(*gd);
    CHECK_EQ(p.size(), size_t(3));
    CHECK_EQ(p[0].bdf, std::string("0000:e8:00.0"));
    CHECK_EQ(p[0].pci_class, uint32_t(0x060400));
    CHECK_EQ(p[1].bdf, std::string("0000:f0:00.0"));
    CHECK_EQ(p[2].bdf, std::string("0000:f2:00.0"));
    auto nd = read_pci_dev(t.path, t.path + "/devices/" + n);
    auto q = rccl_pci_parents(*nd);
    CHECK_EQ(q.size(), size_t(3));
    CHECK_EQ(q[0].bdf, std::string("0000:e8:00.0"));  // shared with the GPU: RCCL's PXB
    CHECK_EQ(q[1].bdf, std::string("0000:ea:00.0"));
    CHECK_EQ(q[2].bdf, std::string("0000:ec:00.0"));
    auto md = read_pci_dev(t.path, t.path + "/devices/" + m);
    CHECK(rccl_pci_parents(*md).empty());  // its parent is the CPU
}

TEST(topology_rccl_link_is_the_slower_of_device_and_port) {
    // NCCL xml.cc: link_speed = the slower of the device's and its port's max_link_speed (as the
    // string read), link_width = the narrower width; missing files read as "" / 0.
    PciDev d;
    d.max_link_speed = "32.0 GT/s PCIe";
    d.port_max_link_speed = "5.0 GT/s PCIe";
    d.max_link_width = 16;
    d.port_max_link_width = 8;
    CHECK_EQ(d.rccl_link_speed(), std::string("5.0 GT/s PCIe"));
    CHECK_EQ(d.rccl_link_width(), 8);
    d.port_max_link_speed = "";
    CHECK_EQ(d.rccl_link_speed(), std::string("32.0 GT/s PCIe"));
    d.max_link_speed = "";
    CHECK_EQ(d.rccl_link_speed(), std::string(""));
    d.port_max_link_width = 0;
    CHECK_EQ(d.rccl_link_width(), 0);
}

TEST(topology_rdma_mode_leaves_the_gpu_rails_to_the_scale_out_agent) {
    // host-nic discovery: every RDMA NIC of the driver list except the GPUs' rails, which the
    // amd-so agent owns; each left-out rail is named with its GPU.
    TmpDir t;
    build_node(t);
    t.mkdir("devices/pci0000:37/0000:37:01.1/0000:38:00.0/infiniband/mlx5_8");
    DiscoveryOptions opt;
    opt.mode = DiscoveryMode::Rdma;
    auto r = discover(opt, t.path);
    CHECK_EQ(r.ifnames.size(), size_t(1));
    CHECK_EQ(r.ifnames[0], std::string("ens9np0"));
    CHECK_EQ(r.excluded.size(), size_t(2));
    CHECK_EQ(r.excluded[0].first, std::string("enp5s0np0"));
    CHECK(r.excluded[0].second.find("scale-out rail of GPU 0000:0a:00.0 (amdgpu, path PXB)") != std::string::npos);
    CHECK_EQ(r.excluded[1].first, std::string("enp30s0np0"));
    opt.exclude_gpu_rails = false;  // --rdma-include-gpu-rails
    auto all = discover(opt, t.path);
    CHECK_EQ(all.ifnames.size(), size_t(3));
    CHECK(all.excluded.empty());
}
