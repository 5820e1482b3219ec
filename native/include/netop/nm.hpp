// Take scale-out interfaces away from NetworkManager.
//
// Reference: internal/nm/networkmanager.go — if reading NM's Version fails, NM is assumed
// absent and nothing is done (:81-86); otherwise every NM device whose Interface is in
// the list gets Managed=false (:88-107).  The interfaces are abstract so tests can inject
// failures (networkmanager_test.go:25-47).  In addition to the runtime D-Bus change we can
// persist the choice as an NM keyfile snippet (unmanaged-devices=interface-name:...), so the
// interfaces stay unmanaged across NetworkManager restarts.
#pragma once

#include <memory>
#include <string>
#include <vector>

namespace netop::nm {

class DeviceIf {
   public:
    virtual ~DeviceIf() = default;
    virtual std::string get_interface() = 0;
    virtual void set_managed(bool managed) = 0;
};

class NetworkManagerIf {
   public:
    virtual ~NetworkManagerIf() = default;
    virtual std::string get_version() = 0;
    virtual std::vector<std::unique_ptr<DeviceIf>> get_all_devices() = 0;
};

// Real implementation over the system bus.  Throws if the bus cannot be reached.
std::unique_ptr<NetworkManagerIf> connect_system_bus(const std::string& address = "");

// Returns the interfaces that were switched to unmanaged.  Throws on device errors.
std::vector<std::string> disable_for_interfaces(NetworkManagerIf& nm, const std::vector<std::string>& ifaces);

// Keyfile snippet for /etc/NetworkManager/conf.d/.  The list is appended to
// ("unmanaged-devices+="), so the files of two agents on one node (an amd-so and a host-nic
// policy) and the host's own setting all apply; a plain "=" in a later file would replace them.
std::string keyfile_snippet(const std::vector<std::string>& ifaces);
// The keyfile's name for an agent publishing `label_file`: 99-amd-network-operator.conf for the
// default scale-out label file, 99-amd-network-operator-<label file stem>.conf otherwise (one
// file per agent, so one agent's teardown never removes another's).
std::string keyfile_name(const std::string& label_file);
// Writes <conf_dir>/<name> if conf_dir's parent exists; returns the path or "".
std::string write_keyfile(const std::string& conf_dir, const std::vector<std::string>& ifaces,
                          const std::string& name = keyfile_name(""));
// Teardown: removes that keyfile if it is ours (starts with the agent's header line), so the NICs
// go back to NetworkManager at its next start.  True when a file was removed.
bool remove_keyfile(const std::string& conf_dir, const std::string& name = keyfile_name(""));
// Teardown of the runtime change: Managed=true again on the named devices NM knows.  Returns the
// interfaces re-managed.  Throws on device errors.
std::vector<std::string> restore_for_interfaces(NetworkManagerIf& nm, const std::vector<std::string>& ifaces);

}  // namespace netop::nm
