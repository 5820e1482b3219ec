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
