"""The agent's C++ D-Bus client against an independent Python implementation of the bus
(NetworkManager impersonation)."""

import pytest

from network_operator_amd.testing.fakedbus import FakeNetworkManagerBus, decode, encode


def test_python_codec_roundtrip():
    b = encode(1, 7, {"path": "/a", "member": "Set", "interface": "i.f", "destination": "d"}, "ssv",
               ("x", "y", ("b", True)))
    m, used = decode(b)
    assert used == len(b) and m["body"] == ["x", "y", ("b", True)] and m["serial"] == 7


def test_disable_networkmanager_for_interfaces(native, tmp_path):
    bus = FakeNetworkManagerBus(str(tmp_path / "bus"), {"ens1": True, "ens2": True, "eth0": True})
    try:
        done = native.nm_disable_interfaces(bus.address, ["ens1", "ens2", "absent"])
        assert sorted(done) == ["ens1", "ens2"]
        assert bus.devices == {"ens1": False, "ens2": False, "eth0": True}
        assert bus.auth_lines[0].startswith("AUTH EXTERNAL ")
        members = [c[2] for c in bus.calls]
        assert members[0] == "Hello" and "GetAllDevices" in members and members.count("Set") == 2
        assert native.dbus_call_get_property(bus.address, "org.freedesktop.NetworkManager",
                                             "/org/freedesktop/NetworkManager", "org.freedesktop.NetworkManager",
                                             "Version") == "1.46.0"
    finally:
        bus.stop()


def test_networkmanager_not_running_is_not_an_error(native, tmp_path):
    bus = FakeNetworkManagerBus(str(tmp_path / "bus"), {"ens1": True}, nm_running=False)
    try:
        assert native.nm_disable_interfaces(bus.address, ["ens1"]) == []
        assert bus.devices["ens1"] is True
    finally:
        bus.stop()


def test_set_managed_failure_propagates(native, tmp_path):
    bus = FakeNetworkManagerBus(str(tmp_path / "bus"), {"ens1": True}, fail_set=True)
    try:
        with pytest.raises(Exception, match="PermissionDenied"):
            native.nm_disable_interfaces(bus.address, ["ens1"])
    finally:
        bus.stop()


def test_no_bus_is_an_error(native, tmp_path):
    with pytest.raises(OSError):
        native.nm_disable_interfaces(f"unix:path={tmp_path}/nothing", ["ens1"])


# ------------------------------------------------------------------------------------------
# The same client against freedesktop's own bus implementation (dbus-daemon), so a misreading
# of the spec shared by the client and the Python fake cannot pass unnoticed.
# ------------------------------------------------------------------------------------------
from network_operator_amd.testing.fakedbus import BusDaemon, NetworkManagerOnBus  # noqa: E402

needs_daemon = pytest.mark.skipif(not BusDaemon.available(), reason="dbus-daemon not installed")


@pytest.fixture
def daemon(tmp_path):
    d = BusDaemon(str(tmp_path))
    yield d
    d.stop()


@needs_daemon
def test_client_talks_to_real_dbus_daemon(native, daemon):
    """SASL EXTERNAL, Hello and marshalling accepted by dbus-daemon (which validates every
    message and disconnects a client that sends a malformed one)."""
    unique, (names,) = native.dbus_call(daemon.address, "org.freedesktop.DBus", "/org/freedesktop/DBus",
                                        "org.freedesktop.DBus", "ListNames")
    assert unique.startswith(":1.") and "org.freedesktop.DBus" in names and unique in names
    _, (bus_id,) = native.dbus_call(daemon.address, "org.freedesktop.DBus", "/org/freedesktop/DBus",
                                    "org.freedesktop.DBus", "GetId")
    assert len(bus_id) == 32 and int(bus_id, 16) >= 0
    assert isinstance(native.dbus_call_get_property(daemon.address, "org.freedesktop.DBus", "/org/freedesktop/DBus",
                                                    "org.freedesktop.DBus", "Features"), list)  # "as" demarshalled
    with pytest.raises(Exception, match="UnknownMethod|ServiceUnknown|AccessDenied"):
        native.dbus_call(daemon.address, "org.freedesktop.DBus", "/org/freedesktop/DBus", "org.freedesktop.DBus",
                         "NoSuchMethod")


@needs_daemon
def test_disable_and_restore_through_real_dbus_daemon(native, daemon):
    nm = NetworkManagerOnBus(daemon.address, {"ens1": True, "ens2": True, "eth0": True})
    try:
        done = native.nm_disable_interfaces(daemon.address, ["ens1", "ens2", "absent"])
        assert sorted(done) == ["ens1", "ens2"]
        assert nm.devices == {"ens1": False, "ens2": False, "eth0": True}
        # Routed by the daemon: the service saw the agent's calls with the daemon's headers.
        assert [c[2] for c in nm.calls].count("Set") == 2
        assert native.dbus_call_get_property(daemon.address, "org.freedesktop.NetworkManager",
                                             "/org/freedesktop/NetworkManager/Devices/1",
                                             "org.freedesktop.NetworkManager.Device", "Managed") is False
        # Teardown hands them back.
        assert sorted(native.nm_restore_interfaces(daemon.address, ["ens1", "ens2"])) == ["ens1", "ens2"]
        assert nm.devices == {"ens1": True, "ens2": True, "eth0": True}
    finally:
        nm.stop()


@needs_daemon
def test_networkmanager_absent_on_real_bus_is_not_an_error(native, daemon):
    # Nobody owns org.freedesktop.NetworkManager: the daemon answers ServiceUnknown and the agent
    # treats NM as not running (reference internal/nm/networkmanager.go:81-86).
    assert native.nm_disable_interfaces(daemon.address, ["ens1"]) == []
