#include "netop/nm.hpp"

#include <unistd.h>

#include <algorithm>
#include <cctype>

#include "netop/common.hpp"
#include "netop/dbus.hpp"
#include "netop/log.hpp"

namespace netop::nm {

namespace {
constexpr const char* kBus = "org.freedesktop.NetworkManager";
constexpr const char* kPath = "/org/freedesktop/NetworkManager";
constexpr const char* kDeviceIface = "org.freedesktop.NetworkManager.Device";

class BusDevice final : public DeviceIf {
   public:
    BusDevice(std::shared_ptr<dbus::Connection> c, std::string path) : c_(std::move(c)), path_(std::move(path)) {}
    std::string get_interface() override { return c_->get_property(kBus, path_, kDeviceIface, "Interface").as_string(); }
    void set_managed(bool managed) override {
        c_->set_property(kBus, path_, kDeviceIface, "Managed", dbus::Value::boolean(managed));
    }

   private:
    std::shared_ptr<dbus::Connection> c_;
    std::string path_;
};

class BusNetworkManager final : public NetworkManagerIf {
   public:
    explicit BusNetworkManager(std::shared_ptr<dbus::Connection> c) : c_(std::move(c)) {}
    std::string get_version() override { return c_->get_property(kBus, kPath, kBus, "Version").as_string(); }
    std::vector<std::unique_ptr<DeviceIf>> get_all_devices() override {
        auto r = c_->call(kBus, kPath, kBus, "GetAllDevices");
        std::vector<std::unique_ptr<DeviceIf>> out;
        if (r.empty()) return out;
        for (const auto& p : r[0].as_array()) out.push_back(std::make_unique<BusDevice>(c_, p.as_string()));
        return out;
    }

   private:
    std::shared_ptr<dbus::Connection> c_;
};
}  // namespace

std::unique_ptr<NetworkManagerIf> connect_system_bus(const std::string& address) {
    auto c = std::make_shared<dbus::Connection>(address.empty() ? dbus::Connection::system_bus_address() : address);
    return std::make_unique<BusNetworkManager>(std::move(c));
}

std::vector<std::string> disable_for_interfaces(NetworkManagerIf& nm, const std::vector<std::string>& ifaces) {
    std::vector<std::string> done;
    try {
        nm.get_version();
    } catch (const std::exception& e) {
        NLOG_I("Couldn't read NetworkManager version. It's probably not running. (%s)", e.what());
        return done;
    }
    for (auto& dev : nm.get_all_devices()) {
        std::string name = dev->get_interface();
        if (std::find(ifaces.begin(), ifaces.end(), name) == ifaces.end()) continue;
        dev->set_managed(false);
        NLOG_I("Disabled NetworkManager for interface %s", name.c_str());
        done.push_back(name);
    }
    return done;
}

static const char* const kKeyfileHeader = "# Written by the AMD network operator: scale-out NICs are configured by its agent.\n";
static const char* const kKeyfileName = "99-amd-network-operator.conf";

std::vector<std::string> restore_for_interfaces(NetworkManagerIf& nm, const std::vector<std::string>& ifaces) {
    std::vector<std::string> done;
    try {
        nm.get_version();
    } catch (const std::exception&) {
        return done;  // NetworkManager gone meanwhile: nothing to give back
    }
    for (auto& dev : nm.get_all_devices()) {
        std::string name = dev->get_interface();
        if (std::find(ifaces.begin(), ifaces.end(), name) == ifaces.end()) continue;
        dev->set_managed(true);
        NLOG_I("Re-enabled NetworkManager for interface %s", name.c_str());
        done.push_back(name);
    }
    return done;
}

std::string keyfile_name(const std::string& label_file) {
    if (label_file.empty() || label_file == "scale-out-readiness.txt") return kKeyfileName;
    std::string stem = label_file.substr(0, label_file.rfind('.'));
    for (char& c : stem)
        if (!std::isalnum(static_cast<unsigned char>(c)) && c != '-' && c != '_') c = '-';
    return "99-amd-network-operator-" + stem + ".conf";
}

bool remove_keyfile(const std::string& conf_dir, const std::string& name) {
    if (conf_dir.empty()) return false;
    std::string path = path_join(conf_dir, name);
    auto s = read_file(path);
    if (!s || s->rfind(kKeyfileHeader, 0) != 0) return false;  // absent, or not written by us
    return ::unlink(path.c_str()) == 0;
}

std::string keyfile_snippet(const std::vector<std::string>& ifaces) {
    std::vector<std::string> items;
    for (auto& i : ifaces) items.push_back("interface-name:" + i);
    return std::string(kKeyfileHeader) +
           "[keyfile]\n"
           "unmanaged-devices+=" +
           join(items, ";") + "\n";
}

std::string write_keyfile(const std::string& conf_dir, const std::vector<std::string>& ifaces,
                          const std::string& name) {
    if (ifaces.empty() || !is_dir(path_dirname(conf_dir))) return "";
    mkdir_p(conf_dir);
    std::string path = path_join(conf_dir, name);
    write_file_atomic(path, keyfile_snippet(ifaces), 0644);
    return path;
}

}  // namespace netop::nm
