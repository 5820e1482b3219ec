#include <sys/stat.h>
#include <unistd.h>

#include "check.hpp"
#include "netop/artifacts.hpp"
#include "tmpdir.hpp"

using namespace netop;
using namespace netop::artifacts;

static NicState nic(const std::string& name, const char* mac, const char* peer_desc, const char* peer_mac, int gpu = -1) {
    NicState n;
    n.ifname = name;
    n.link.name = name;
    n.link.index = 7;
    n.link.mac = *MacAddr::parse(mac);
    if (peer_desc) n.addr = l3::parse_port_description(peer_desc, l3::TokenPolicy::Compat, nullptr);
    if (peer_mac) n.peer_mac = MacAddr::parse(peer_mac);
    n.gpu_index = gpu;
    return n;
}

TEST(rccl_net_legacy_golden) {
    // Same entry schema and key order as the reference's gaudinet.json golden
    // (reference cmd/discover/gaudinet_test.go:42-44).
    std::vector<NicState> v{nic("eth1234", "01:02:03:04:05:06", "x 10.120.0.2/30", "06:05:04:03:02:01")};
    CHECK_EQ(generate_rccl_net(v, false),
             std::string("{\"NIC_NET_CONFIG\":[{\"NIC_MAC\":\"01:02:03:04:05:06\","
                         "\"NIC_IP\":\"10.120.0.1\",\"SUBNET_MASK\":\"255.255.255.252\","
                         "\"GATEWAY_MAC\":\"06:05:04:03:02:01\"}]}"));
}

TEST(rccl_net_extended_and_skips) {
    auto a = nic("ens1", "02:00:00:00:00:01", "x 10.0.0.2/30", "02:00:00:00:01:01", 1);
    a.gpu_bdf = "0000:23:00.0";
    a.rdma_dev = "mlx5_3";
    a.gid_index = 3;
    auto b = nic("ens0", "02:00:00:00:00:02", "x 10.0.0.6/30", "02:00:00:00:01:02", 0);
    auto no_addr = nic("ens2", "02:00:00:00:00:03", nullptr, "02:00:00:00:01:03", 2);
    auto no_peer = nic("ens3", "02:00:00:00:00:04", "x 10.0.0.10/30", nullptr, 3);
    std::string j = generate_rccl_net({a, b, no_addr, no_peer});
    // Sorted by GPU index: ens0 (gpu 0) before ens1 (gpu 1); ens2/ens3 skipped.
    CHECK(j.find("ens0") < j.find("ens1"));
    CHECK(j.find("ens2") == std::string::npos);
    CHECK(j.find("ens3") == std::string::npos);
    CHECK(j.find("\"GPU_BDF\":\"0000:23:00.0\"") != std::string::npos);
    CHECK(j.find("\"RDMA_DEV\":\"mlx5_3\",\"RDMA_PORT\":1,\"GID_INDEX\":3") != std::string::npos);
    CHECK(j.find("\"GATEWAY_IP\":\"10.0.0.6\"") != std::string::npos);
    CHECK_EQ(generate_rccl_net({}), std::string("{\"NIC_NET_CONFIG\":[]}"));
}

TEST(rccl_net_write_mode_and_errors) {
    TmpDir t;
    std::string p = t.path + "/rccl-net.json";
    write_rccl_net(p, {nic("eth0", "01:02:03:04:05:06", "x 10.210.8.121/30", "01:02:03:04:05:07")});
    struct stat st;
    CHECK(::stat(p.c_str(), &st) == 0);
    CHECK_EQ(int(st.st_mode & 0777), 0644);
    CHECK_THROWS(write_rccl_net("", {}));
    CHECK_THROWS(write_rccl_net(t.path + "/missing/dir/x.json", {}));
}

TEST(rccl_env_contents) {
    auto a = nic("ens1", "02:00:00:00:00:01", "x 10.0.0.2/30", "02:00:00:00:01:01", 1);
    a.rdma_dev = "mlx5_3";
    a.configured = true;
    a.gid_index = 3;
    auto b = nic("ens0", "02:00:00:00:00:02", "x 10.0.0.6/30", "02:00:00:00:01:02", 0);
    b.rdma_dev = "mlx5_1";
    b.configured = true;
    b.gid_index = 3;
    auto env = generate_rccl_env({a, b}, "/etc/amd/scale-out/rccl-topo.xml");
    CHECK(env.find("NCCL_IB_HCA==mlx5_1:1,mlx5_3:1\n") != std::string::npos);
    CHECK(env.find("NCCL_IB_GID_INDEX=3\n") != std::string::npos);
    CHECK(env.find("NCCL_TOPO_FILE=/etc/amd/scale-out/rccl-topo.xml\n") != std::string::npos);
    CHECK(env.find("NCCL_IB_ADDR_FAMILY") == std::string::npos);
    b.gid_index = 5;  // inconsistent GID indices: steer RCCL's own per-NIC selection instead
    env = generate_rccl_env({a, b}, "");
    CHECK(env.find("NCCL_IB_GID_INDEX") == std::string::npos);
    CHECK(env.find("NCCL_IB_ROCE_VERSION_NUM=2\nNCCL_IB_ADDR_FAMILY=AF_INET\n") != std::string::npos);
    b.gid_index.reset();  // one GID not found yet: never pin the other NIC's index for both
    env = generate_rccl_env({a, b}, "", {}, {}, true);
    CHECK(env.find("NCCL_IB_GID_INDEX") == std::string::npos);
    CHECK(env.find("NCCL_IB_ADDR_FAMILY=AF_INET6\n") != std::string::npos);
}

TEST(networkd_golden_and_rollback) {
    // Golden text of the reference (cmd/discover/systemd-networkd_test.go:76-86).
    auto n = nic("eth0", "01:02:03:04:05:06", "x 10.210.8.121/30", "01:02:03:04:05:07");
    CHECK_EQ(generate_networkd(n), std::string("[Match]\n"
                                               "MACAddress=01:02:03:04:05:06\n"
                                               "\n"
                                               "[Network]\n"
                                               "Description=Networkd configuration for eth0 created by network-operator\n"
                                               "Address=10.210.8.122/30\n"
                                               "\n"
                                               "[Route]\n"
                                               "Destination=10.210.0.0/16\n"));
    TmpDir t;
    auto written = write_networkd(t.path, {n});
    CHECK_EQ(written.size(), size_t(1));
    CHECK(path_exists(t.path + "/eth0.network"));
    // Validation happens before any write: missing address -> nothing written.
    auto bad = nic("eth1", "01:02:03:04:05:08", nullptr, nullptr);
    CHECK_THROWS(write_networkd(t.path, {bad}));
    CHECK(!path_exists(t.path + "/eth1.network"));
    auto nomac = nic("eth2", "00:00:00:00:00:00", "x 10.0.0.2/30", nullptr);
    CHECK_THROWS(write_networkd(t.path, {nomac}));
    CHECK_THROWS(write_networkd(t.path + "/nope", {n}));
    delete_networkd(t.path, written);
    CHECK(!path_exists(t.path + "/eth0.network"));
}

TEST(labels_written_only_with_features_dir) {
    TmpDir t;
    Labels l;
    l.dir = t.path + "/features.d";
    CHECK(!write_labels(l, {}));
    ::mkdir(l.dir.c_str(), 0755);
    CHECK(write_labels(l, {{"amd.feature.node.kubernetes.io/gpu-scale-out.nics", "8"}}));
    auto s = read_file(l.path());
    CHECK_EQ(*s, std::string("amd.feature.node.kubernetes.io/gpu-scale-out=true\n"
                             "amd.feature.node.kubernetes.io/gpu-scale-out.nics=8\n"));
    CHECK(remove_labels(l));
    CHECK(!path_exists(l.path()));
}

TEST(json_escaping) {
    Json j;
    j.begin_object().key("a\"b").value(std::string("x<y>&\n\x01")).key("n").value(int64_t(-3)).key("d").value(0.5);
    j.key("arr").begin_array().value(true).null().end_array().end_object();
    CHECK_EQ(j.str(), std::string("{\"a\\\"b\":\"x\\u003cy\\u003e\\u0026\\n\\u0001\",\"n\":-3,\"d\":0.5,\"arr\":[true,null]}"));
}

TEST(rccl_env_extra_settings) {
    auto ex = parse_env_extra("NCCL_IB_TC=106, NCCL_IB_QPS_PER_CONNECTION=4,HSA_NO_SCRATCH_RECLAIM=1");
    CHECK_EQ(ex.size(), size_t(3));
    NicState a;
    a.ifname = "e0";
    a.rdma_dev = "mlx5_0";
    a.configured = true;
    auto env = generate_rccl_env({a}, "", ex);
    CHECK(env.find("NCCL_IB_TC=106\n") != std::string::npos);
    CHECK(env.find("HSA_NO_SCRATCH_RECLAIM=1\n") != std::string::npos);
    CHECK_THROWS(parse_env_extra("PATH=/tmp"));
    CHECK_THROWS(parse_env_extra("NCCL_x=1"));
    CHECK_THROWS(parse_env_extra("NCCL_IB_TC"));
    CHECK(parse_env_extra("").empty());
}

TEST(rccl_topo_xml_tree) {
    TmpDir t;
    auto dev = [&](const std::string& path, const char* cls, const char* vendor, const char* device, int numa) {
        t.mkdir("devices/" + path);
        t.write("devices/" + path + "/class", std::string(cls) + "\n");
        t.write("devices/" + path + "/vendor", std::string(vendor) + "\n");
        t.write("devices/" + path + "/device", std::string(device) + "\n");
        t.write("devices/" + path + "/subsystem_vendor", std::string(vendor) + "\n");
        t.write("devices/" + path + "/subsystem_device", std::string(device) + "\n");
        t.write("devices/" + path + "/numa_node", std::to_string(numa) + "\n");
    };
    const std::string rp = "pci0000:e7/0000:e7:01.1/0000:e8:00.0";
    dev(rp, "0x060400", "0x1000", "0xc030", 1);
    dev(rp + "/0000:e9:08.0/0000:f0:00.0", "0x060400", "0x1000", "0xc030", 1);
    dev(rp + "/0000:e9:08.0/0000:f0:00.0/0000:f1:10.0/0000:f2:00.0", "0x060400", "0x1022", "0x1500", 1);
    const std::string g = rp + "/0000:e9:08.0/0000:f0:00.0/0000:f1:10.0/0000:f2:00.0/0000:f3:00.0/0000:f4:00.0";
    dev(g, "0x120000", "0x1002", "0x75a3", 1);
    dev(rp + "/0000:e9:00.0/0000:ea:00.0", "0x060400", "0x1000", "0xc030", 1);
    dev(rp + "/0000:e9:00.0/0000:ea:00.0/0000:eb:10.0/0000:ec:00.0", "0x060400", "0x1000", "0xc030", 1);
    const std::string n = rp + "/0000:e9:00.0/0000:ea:00.0/0000:eb:10.0/0000:ec:00.0/0000:ed:01.0/0000:ef:00.0";
    dev(n, "0x020000", "0x15b3", "0x1021", 1);
    topo::Gpu gpu;
    gpu.pci = *topo::read_pci_dev(t.path, t.path + "/devices/" + g);
    TopoNic tn;
    tn.pci = *topo::read_pci_dev(t.path, t.path + "/devices/" + n);
    tn.net_name = "mlx5_7";
    tn.port = 1;
    t.write("devices/system/node/node1/cpumap", "ffffffff,00000000\n");
    topo::CpuIdentity cpu{"x86_64", "AuthenticAMD", 191, 2};
    std::string x = generate_rccl_topo({gpu}, {tn}, cpu, t.path);
    const std::string want =
        "<system version=\"2\">\n"
        "  <cpu numaid=\"1\" affinity=\"ffffffff,00000000\" arch=\"x86_64\" vendor=\"AuthenticAMD\" familyid=\"191\" modelid=\"2\">\n"
        "    <pci busid=\"0000:e8:00.0\" class=\"0x060400\" vendor=\"0x1000\" device=\"0xc030\" subsystem_vendor=\"0x1000\" subsystem_device=\"0xc030\" link_speed=\"\" link_width=\"0\">\n"
        "      <pci busid=\"0000:ea:00.0\" class=\"0x060400\" vendor=\"0x1000\" device=\"0xc030\" subsystem_vendor=\"0x1000\" subsystem_device=\"0xc030\" link_speed=\"\" link_width=\"0\">\n"
        "        <pci busid=\"0000:ec:00.0\" class=\"0x060400\" vendor=\"0x1000\" device=\"0xc030\" subsystem_vendor=\"0x1000\" subsystem_device=\"0xc030\" link_speed=\"\" link_width=\"0\">\n"
        "          <pci busid=\"0000:ef:00.0\" class=\"0x020000\" vendor=\"0x15b3\" device=\"0x1021\" subsystem_vendor=\"0x15b3\" subsystem_device=\"0x1021\" link_speed=\"\" link_width=\"0\">\n"
        "            <nic>\n"
        "              <net name=\"mlx5_7\" port=\"1\"/>\n"
        "            </nic>\n"
        "          </pci>\n"
        "        </pci>\n"
        "      </pci>\n"
        "      <pci busid=\"0000:f0:00.0\" class=\"0x060400\" vendor=\"0x1000\" device=\"0xc030\" subsystem_vendor=\"0x1000\" subsystem_device=\"0xc030\" link_speed=\"\" link_width=\"0\">\n"
        "        <pci busid=\"0000:f2:00.0\" class=\"0x060400\" vendor=\"0x1022\" device=\"0x1500\" subsystem_vendor=\"0x1022\" subsystem_device=\"0x1500\" link_speed=\"\" link_width=\"0\">\n"
        "          <pci busid=\"0000:f4:00.0\" class=\"0x120000\" vendor=\"0x1002\" device=\"0x75a3\" subsystem_vendor=\"0x1002\" subsystem_device=\"0x75a3\" link_speed=\"\" link_width=\"0\"/>\n"
        "        </pci>\n"
        "      </pci>\n"
        "    </pci>\n"
        "  </cpu>\n"
        "</system>\n";
    CHECK_EQ(x, want);
    // rccl.env points RCCL at it and pins the socket interfaces.
    auto a = nic("enp239s0np0", "02:00:00:00:00:01", "x 10.0.0.2/30", "02:00:00:00:01:01", 7);
    auto env = generate_rccl_env({a}, "/etc/amd/scale-out/rccl-topo.xml", {}, {"enp239s0np0", "enp8s0np0"});
    CHECK(env.find("NCCL_TOPO_FILE=/etc/amd/scale-out/rccl-topo.xml\n") != std::string::npos);
    CHECK(env.find("NCCL_SOCKET_IFNAME==enp239s0np0,enp8s0np0\n") != std::string::npos);
}
