// pybind11 module `_netop_native`: exposes the agent's native building blocks to Python
// for the netns integration harness, the fake-sysfs topology tests and property-based
// (hypothesis) fuzzing of the LLDP codec / Port-Description parser.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/socket.h>

#include "netop/agent.hpp"
#include "netop/artifacts.hpp"
#include "netop/dbus.hpp"
#include "netop/l3.hpp"
#include "netop/lldp.hpp"
#include "netop/netlink.hpp"
#include "netop/nm.hpp"
#include "netop/packet.hpp"
#include "netop/topology.hpp"

namespace py = pybind11;
using namespace netop;

static MacAddr mac_of(const std::string& s) {
    auto m = MacAddr::parse(s);
    if (!m) throw py::value_error("bad MAC address '" + s + "'");
    return *m;
}

static py::dict link_dict(const nl::LinkInfo& l) {
    py::dict d;
    d["index"] = l.index;
    d["name"] = l.name;
    d["flags"] = l.flags;
    d["up"] = l.up();
    d["mtu"] = l.mtu;
    d["mac"] = l.mac.str();
    d["operstate"] = l.operstate_str();
    d["kind"] = l.kind;
    d["master"] = l.master;
    return d;
}

static py::dict frame_dict(const lldp::Frame& f) {
    py::dict d;
    d["dst"] = f.dst.str();
    d["src"] = f.src.str();
    d["chassis_subtype"] = f.chassis_subtype;
    d["chassis_id"] = py::bytes(f.chassis_id);
    d["port_subtype"] = f.port_subtype;
    d["port_id"] = py::bytes(f.port_id);
    d["ttl"] = f.ttl;
    d["port_description"] = f.port_description ? py::object(py::str(*f.port_description)) : py::none();
    d["system_name"] = f.system_name ? py::object(py::str(*f.system_name)) : py::none();
    d["system_description"] = f.system_description ? py::object(py::str(*f.system_description)) : py::none();
    auto pm = f.peer_mac();
    d["peer_mac"] = pm ? py::object(py::str(pm->str())) : py::none();
    d["vlan"] = f.vlan ? py::object(py::int_(*f.vlan)) : py::none();
    d["management"] = py::int_(f.management.size());
    d["org"] = py::int_(f.org.size());
    return d;
}

// Demarshalled D-Bus value -> Python (strings, booleans, integers, arrays / structs as lists).
static py::object dbus_to_py(const dbus::Value& v) {
    const char c = v.sig.empty() ? '?' : v.sig[0];
    if (c == 's' || c == 'o' || c == 'g') return py::str(v.as_string());
    if (c == 'b') return py::bool_(v.as_bool());
    if (c == 'v') return dbus_to_py(v.variant_inner());
    if (c == 'a' || c == '(') {
        py::list l;
        for (auto& x : v.as_array()) l.append(dbus_to_py(x));
        return l;
    }
    if (auto p = std::get_if<uint32_t>(&v.v)) return py::int_(*p);
    if (auto p = std::get_if<int32_t>(&v.v)) return py::int_(*p);
    if (auto p = std::get_if<uint8_t>(&v.v)) return py::int_(*p);
    if (auto p = std::get_if<int64_t>(&v.v)) return py::int_(*p);
    if (auto p = std::get_if<uint64_t>(&v.v)) return py::int_(*p);
    return py::str("<" + v.sig + ">");
}

PYBIND11_MODULE(_netop_native, m) {
    m.doc() = "Native building blocks of the AMD MI355X network operator agent";
    m.attr("__version__") = NETOP_VERSION;

    py::register_exception<SysError>(m, "SysError", PyExc_OSError);

    // ---- LLDP -------------------------------------------------------------
    m.def("lldp_switch_frame", [](const std::string& mac, const std::string& sysname, const std::string& port,
                                  const std::string& desc, int ttl, py::object vlan) {
        auto f = lldp::make_switch_frame(mac_of(mac), sysname, port, desc, uint16_t(ttl));
        if (!vlan.is_none()) f.vlan = uint16_t(vlan.cast<int>());
        auto b = lldp::encode(f);
        return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
    }, py::arg("mac"), py::arg("system_name"), py::arg("port"), py::arg("port_description"), py::arg("ttl") = 120,
       py::arg("vlan") = py::none());
    m.def("lldp_encode", [](const std::string& src, int chassis_subtype, const py::bytes& chassis_id, int port_subtype,
                            const py::bytes& port_id, int ttl, py::object port_desc, py::object sysname) {
        lldp::Frame f;
        f.src = mac_of(src);
        f.chassis_subtype = uint8_t(chassis_subtype);
        f.chassis_id = std::string(chassis_id);
        f.port_subtype = uint8_t(port_subtype);
        f.port_id = std::string(port_id);
        f.ttl = uint16_t(ttl);
        if (!port_desc.is_none()) f.port_description = port_desc.cast<std::string>();
        if (!sysname.is_none()) f.system_name = sysname.cast<std::string>();
        auto b = lldp::encode(f);
        return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
    }, py::arg("src"), py::arg("chassis_subtype"), py::arg("chassis_id"), py::arg("port_subtype"), py::arg("port_id"),
       py::arg("ttl") = 120, py::arg("port_description") = py::none(), py::arg("system_name") = py::none());
    m.def("lldp_decode", [](const py::bytes& data) -> py::object {
        std::string s(data);
        lldp::DecodeError e;
        auto f = lldp::decode(reinterpret_cast<const uint8_t*>(s.data()), s.size(), &e);
        if (!f) throw py::value_error(lldp::to_string(e));
        return frame_dict(*f);
    });

    // ---- L3 ---------------------------------------------------------------
    // The agent's regular-expression dialect (ECMAScript std::regex), for the webhook's tests.
    m.def("ecmascript_regex_error", &agent::ecmascript_regex_error);
    m.def("ecmascript_full_match", &agent::ecmascript_full_match);
    m.def("rail_pattern_error", &agent::rail_pattern_error);
    m.def("parse_port_description", [](const std::string& desc, const std::string& policy) -> py::object {
        auto p = l3::parse_token_policy(policy);
        if (!p) throw py::value_error("bad token policy");
        std::string err;
        auto a = l3::parse_port_description(desc, *p, &err);
        if (!a) throw py::value_error(err);
        py::dict d;
        d["peer"] = a->peer.str();
        d["local"] = a->local.str();
        d["prefix"] = a->prefix;
        d["p2p_network"] = a->p2p_network().str();
        d["routed_network"] = a->routed_network().str();
        return d;
    }, py::arg("description"), py::arg("policy") = "compat-then-last");

    // ---- rtnetlink ----------------------------------------------------------
    py::class_<nl::Rtnl>(m, "Rtnl")
        .def(py::init<>())
        .def("link_by_name", [](nl::Rtnl& r, const std::string& n) { return link_dict(r.link_by_name(n)); })
        .def("link_list", [](nl::Rtnl& r) {
            py::list l;
            for (auto& x : r.link_list()) l.append(link_dict(x));
            return l;
        })
        .def("addr_list", [](nl::Rtnl& r, int ifindex) {
            py::list l;
            for (auto& a : r.addr_list(ifindex, AF_INET)) l.append(a.prefix().str());
            return l;
        }, py::arg("ifindex") = 0)
        .def("addr6_list", [](nl::Rtnl& r, int ifindex) {
            py::list l;
            for (auto& a : r.addr_list(ifindex, AF_INET6)) {
                py::dict d;
                d["address"] = a.address6;
                d["prefixlen"] = a.prefixlen;
                d["scope"] = int(a.scope);
                d["ifindex"] = a.ifindex;
                l.append(d);
            }
            return l;
        }, py::arg("ifindex") = 0)
        .def("addr_add", [](nl::Rtnl& r, int ifindex, const std::string& cidr) {
            auto p = Ipv4Prefix::parse(cidr);
            if (!p) throw py::value_error("bad CIDR");
            r.addr_add(ifindex, *p);
        })
        .def("addr_del", [](nl::Rtnl& r, int ifindex, const std::string& cidr) {
            auto p = Ipv4Prefix::parse(cidr);
            if (!p) throw py::value_error("bad CIDR");
            for (const auto& a : r.addr_list(ifindex, AF_INET))
                if (a.local == p->addr && a.prefixlen == p->len) {
                    r.addr_del(a);
                    return;
                }
            throw py::value_error("no such address");
        })
        .def("rule_list", [](nl::Rtnl& r) {
            py::list l;
            for (auto& x : r.rule_list()) {
                py::dict d;
                d["src"] = x.src.masked().str();
                d["table"] = x.table;
                d["priority"] = x.priority;
                d["protocol"] = x.protocol;
                d["selective"] = x.selective;
                l.append(d);
            }
            return l;
        })
        .def("route_list", [](nl::Rtnl& r, int table) {
            py::list l;
            for (auto& x : r.route_list(uint32_t(table))) {
                py::dict d;
                d["dst"] = x.dst.masked().str();
                d["gateway"] = x.gateway ? py::object(py::str(x.gateway->str())) : py::none();
                d["prefsrc"] = x.prefsrc ? py::object(py::str(x.prefsrc->str())) : py::none();
                d["ifindex"] = x.ifindex;
                d["protocol"] = x.protocol;
                d["scope"] = x.scope;
                d["table"] = x.table;
                l.append(d);
            }
            return l;
        }, py::arg("table") = int(RT_TABLE_MAIN))
        .def("rule_add", [](nl::Rtnl& r, const std::string& src, uint32_t table, uint32_t priority) {
            nl::RuleSpec rs;
            auto s = Ipv4Prefix::parse(src);
            if (!s) throw py::value_error("bad CIDR");
            rs.src = *s;
            rs.table = table;
            rs.priority = priority;
            r.rule_add(rs);
        }, py::arg("src"), py::arg("table"), py::arg("priority"))
        .def("route_append", [](nl::Rtnl& r, const std::string& dst, py::object gateway, int ifindex, int protocol,
                                uint32_t table) {
            nl::RouteSpec rs;
            auto d = Ipv4Prefix::parse(dst);
            if (!d) throw py::value_error("bad CIDR");
            rs.dst = *d;
            if (!gateway.is_none()) {
                auto g = Ipv4::parse(gateway.cast<std::string>());
                if (!g) throw py::value_error("bad gateway");
                rs.gateway = *g;
            }
            rs.ifindex = ifindex;
            rs.protocol = uint8_t(protocol);
            rs.table = table;
            r.route_append(rs);
        }, py::arg("dst"), py::arg("gateway") = py::none(), py::arg("ifindex") = 0, py::arg("protocol") = int(RTPROT_BOOT),
           py::arg("table") = uint32_t(RT_TABLE_MAIN))
        .def("default_route_links", &nl::Rtnl::default_route_links)
        .def("link_set_up", &nl::Rtnl::link_set_up)
        .def("link_set_down", &nl::Rtnl::link_set_down)
        .def("link_set_mtu", &nl::Rtnl::link_set_mtu)
        .def("link_set_mac", [](nl::Rtnl& r, int idx, const std::string& mac) { r.link_set_mac(idx, mac_of(mac)); })
        .def("veth_add", &nl::Rtnl::veth_add)
        .def("link_add", &nl::Rtnl::link_add, py::arg("name"), py::arg("kind"))
        .def("link_set_master", &nl::Rtnl::link_set_master, py::arg("ifindex"), py::arg("master"))
        .def("link_del", &nl::Rtnl::link_del)
        .def("link_set_netns_pid", &nl::Rtnl::link_set_netns_pid)
        .def("link_set_netns_fd", &nl::Rtnl::link_set_netns_fd)
        .def("link_set_name", &nl::Rtnl::link_set_name)
        .def("dcbx_mode", &nl::Rtnl::dcbx_mode)
        .def("set_dcbx_mode", &nl::Rtnl::set_dcbx_mode)
        .def("round_trips", &nl::Rtnl::round_trips);

    m.def("lldp_send", [](const std::string& ifname, const py::bytes& frame) {
        nl::Rtnl r;
        auto l = r.link_by_name(ifname);
        pkt::LldpSocket s(ifname, l.index, l.mac, false);
        std::string b(frame);
        s.send(std::vector<uint8_t>(b.begin(), b.end()));
    });

    // ---- topology -----------------------------------------------------------
    m.def("discover", [](const std::string& root, const std::string& mode, py::object drivers, const std::string& accel,
                         bool include_gpu_rails) {
        topo::DiscoveryOptions o;
        auto md = topo::parse_discovery_mode(mode);
        if (!md) throw py::value_error("bad mode");
        o.mode = *md;
        o.accel_driver = accel;
        o.exclude_gpu_rails = !include_gpu_rails;
        if (!drivers.is_none()) o.nic_drivers = drivers.cast<std::vector<std::string>>();
        auto r = topo::discover(o, root);
        py::dict d;
        py::list gpus, nics, pairs;
        for (auto& g : r.gpus) {
            py::dict x;
            x["index"] = g.index;
            x["bdf"] = g.pci.bdf;
            x["device"] = g.pci.device;
            x["numa"] = g.pci.numa;
            gpus.append(x);
        }
        for (auto& n : r.nics) {
            py::dict x;
            x["ifname"] = n.ifname;
            x["bdf"] = n.pci.bdf;
            x["driver"] = n.pci.driver;
            x["rdma_dev"] = n.rdma_dev;
            x["mac"] = n.mac.str();
            nics.append(x);
        }
        for (auto& p : r.pairs) {
            py::dict x;
            x["gpu"] = r.gpus[size_t(p.gpu)].pci.bdf;
            x["nic"] = r.nics[size_t(p.nic)].ifname;
            x["path"] = topo::to_string(p.path);
            x["common_depth"] = p.common_depth;
            pairs.append(x);
        }
        d["gpus"] = gpus;
        d["nics"] = nics;
        d["pairs"] = pairs;
        d["ifnames"] = r.ifnames;
        py::dict excluded;
        for (auto& [n, why] : r.excluded) excluded[py::str(n)] = why;
        d["excluded"] = excluded;
        return d;
    }, py::arg("root"), py::arg("mode") = "affine", py::arg("drivers") = py::none(), py::arg("accel_driver") = "amdgpu",
       py::arg("include_gpu_rails") = false);
    m.def("rccl_topo_xml", [](const std::string& root, const std::string& mode, py::object interfaces, int version,
                              py::object cpu) {
        topo::DiscoveryOptions o;
        auto md = topo::parse_discovery_mode(mode);
        if (!md) throw py::value_error("bad mode");
        o.mode = *md;
        auto d = topo::discover(o, root);
        std::vector<std::string> names = d.ifnames;
        if (!interfaces.is_none())
            for (auto& i : interfaces.cast<std::vector<std::string>>())
                if (std::find(names.begin(), names.end(), i) == names.end()) names.push_back(i);
        topo::CpuIdentity id = topo::cpu_identity();
        if (!cpu.is_none()) {  // tests: a fixed identity instead of this machine's CPUID
            auto c = cpu.cast<py::dict>();
            id.arch = c["arch"].cast<std::string>();
            id.vendor = c["vendor"].cast<std::string>();
            id.family = c["family"].cast<int>();
            id.model = c["model"].cast<int>();
        }
        return artifacts::generate_rccl_topo(d.gpus, artifacts::topo_nics(d, names, root), id, root, version);
    }, py::arg("root"), py::arg("mode") = "affine", py::arg("interfaces") = py::none(),
       py::arg("version") = artifacts::kRcclTopoXmlVersion, py::arg("cpu") = py::none());
    m.def("cpu_identity", [] {
        auto c = topo::cpu_identity();
        py::dict d;
        d["arch"] = c.arch;
        d["vendor"] = c.vendor;
        d["family"] = c.family;
        d["model"] = c.model;
        return d;
    });
    m.def("read_xgmi", [](const std::string& root) {
        auto x = topo::read_xgmi(root);
        py::dict d;
        py::list g;
        for (auto& n : x.gpus) g.append(n.bdf());
        d["gpus"] = g;
        d["links"] = x.links.size();
        d["pairs_expected"] = x.pairs_expected;
        d["pairs_connected"] = x.pairs_connected;
        d["full_mesh"] = x.full_mesh();
        d["min_link_bw_mbs"] = x.min_link_bw_mbs;
        d["per_gpu_bw_mbs"] = x.per_gpu_bw_mbs();
        py::list miss;
        for (auto& [a, b] : x.missing) miss.append(py::make_tuple(a, b));
        d["missing"] = miss;
        return d;
    });
    m.def("read_pcie_link", [](const std::string& root, const std::string& bdf) {
        auto l = topo::read_pcie_link(root, bdf);
        py::dict d;
        d["speed_gts"] = l.speed_gts;
        d["max_speed_gts"] = l.max_speed_gts;
        d["width"] = l.width;
        d["max_width"] = l.max_width;
        d["known"] = l.known();
        d["degraded"] = l.degraded();
        d["str"] = l.str();
        return d;
    });
    // timeout_ms > 0: the agent's bounded read (one thread per GPU, late GPUs reported "late").
    m.def("read_xgmi_health", [](const std::string& root, const std::vector<std::string>& bdfs, int64_t timeout_ms) {
        py::list out;
        std::vector<topo::XgmiLinkHealth> hs;
        {
            py::gil_scoped_release nogil;
            hs = timeout_ms > 0 ? topo::read_xgmi_health(root, bdfs, timeout_ms * 1000000) : topo::read_xgmi_health(root, bdfs);
        }
        for (const auto& h : hs) {
            py::dict d;
            d["bdf"] = h.bdf;
            d["revision"] = h.revision;
            d["known"] = h.known;
            d["late"] = h.late;
            d["error"] = h.error;
            d["width"] = h.width;
            d["speed_gbps"] = h.speed_gbps;
            d["status"] = h.status;
            d["read_kb"] = h.read_kb;
            d["write_kb"] = h.write_kb;
            out.append(d);
        }
        return out;
    }, py::arg("root"), py::arg("bdfs"), py::arg("timeout_ms") = 0);
    m.def("detect_gdr", [](const std::string& root, const std::string& kernel) {
        auto g = topo::detect_gdr(root, kernel);
        py::dict d;
        d["mode"] = g.mode();
        d["peer_mem"] = g.peer_mem;
        d["peer_mem_version"] = g.peer_mem_version;
        d["ib_uverbs"] = g.ib_uverbs;
        d["dmabuf"] = g.dmabuf;
        d["kernel"] = g.kernel;
        return d;
    }, py::arg("root") = "/sys/", py::arg("kernel") = "");
    // ---- NetworkManager over the D-Bus wire client ------------------------------------
    // The GIL is released: the peer may be a Python thread in this process (tests).
    m.def("nm_disable_interfaces", [](const std::string& address, const std::vector<std::string>& ifaces) {
        py::gil_scoped_release nogil;
        auto nm = nm::connect_system_bus(address);
        return nm::disable_for_interfaces(*nm, ifaces);
    }, py::arg("address"), py::arg("interfaces"));
    m.def("nm_restore_interfaces", [](const std::string& address, const std::vector<std::string>& ifaces) {
        py::gil_scoped_release nogil;
        auto nm = nm::connect_system_bus(address);
        return nm::restore_for_interfaces(*nm, ifaces);
    }, py::arg("address"), py::arg("interfaces"));
    m.def("dbus_call_get_property", [](const std::string& address, const std::string& dest, const std::string& path,
                                       const std::string& iface, const std::string& prop) {
        dbus::Value v;
        {
            py::gil_scoped_release nogil;
            dbus::Connection c(address);
            v = c.get_property(dest, path, iface, prop);
        }
        return dbus_to_py(v);
    });
    m.def("dbus_call", [](const std::string& address, const std::string& dest, const std::string& path,
                          const std::string& iface, const std::string& member) {
        std::vector<dbus::Value> out;
        std::string unique;
        {
            py::gil_scoped_release nogil;
            dbus::Connection c(address);
            unique = c.unique_name();
            out = c.call(dest, path, iface, member);
        }
        py::list l;
        for (auto& v : out) l.append(dbus_to_py(v));
        return py::make_tuple(unique, l);
    });

    m.def("find_rocev2_gid_index", [](const std::string& root, const std::string& dev, int port, const std::string& ip) -> py::object {
        auto a = Ipv4::parse(ip);
        if (!a) throw py::value_error("bad IPv4");
        auto r = topo::find_rocev2_gid_index(root, dev, port, *a);
        return r ? py::object(py::int_(*r)) : py::none();
    });

}
