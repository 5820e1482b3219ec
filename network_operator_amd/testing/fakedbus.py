"""NetworkManager over D-Bus for the agent's tests: a fake bus and a service on a real bus.

``FakeNetworkManagerBus`` is an independent Python implementation of the protocol subset the
agent's C++ client uses. It covers SASL EXTERNAL, Hello, method calls / returns / errors, and
little-endian marshalling of s o g b u i y v a(). It serves the client directly, as if it were
the bus, so the client is checked against a second implementation rather than against itself.

A second implementation by the same author can share a misreading of the specification. So
``BusDaemon`` also starts the real reference implementation, ``dbus-daemon``, on a private
socket. ``NetworkManagerOnBus`` then joins it as an ordinary client that owns
``org.freedesktop.NetworkManager``. The agent's client has to authenticate to the real daemon and
pass its message validation. Its calls are routed to the service with the daemon's sender and
destination headers. This is the reference's "needs a real system D-Bus" test
(reference internal/nm/networkmanager_test.go:49-62) without needing the host's bus.
"""

from __future__ import annotations

import os
import shutil
import socket
import struct
import subprocess
import threading
from pathlib import Path
from typing import Dict, List, Optional, Tuple


# ---------------------------------------------------------------------------
# marshalling
# ---------------------------------------------------------------------------
def _split(sig: str) -> List[str]:
    out, i = [], 0
    while i < len(sig):
        j = _end(sig, i)
        out.append(sig[i:j])
        i = j
    return out


def _end(sig: str, i: int) -> int:
    c = sig[i]
    if c == "a":
        return _end(sig, i + 1)
    if c in "({":
        close = ")" if c == "(" else "}"
        i += 1
        while sig[i] != close:
            i = _end(sig, i)
        return i + 1
    return i + 1


_ALIGN = {"y": 1, "g": 1, "v": 1, "b": 4, "i": 4, "u": 4, "s": 4, "o": 4, "a": 4, "(": 8, "{": 8, "x": 8, "t": 8}


class W:
    def __init__(self):
        self.b = bytearray()

    def pad(self, n):
        while len(self.b) % n:
            self.b.append(0)

    def put(self, t: str, v):
        c = t[0]
        if c == "y":
            self.b.append(v)
        elif c in "bu":
            self.pad(4)
            self.b += struct.pack("<I", int(v))
        elif c == "i":
            self.pad(4)
            self.b += struct.pack("<i", v)
        elif c in "so":
            self.pad(4)
            e = v.encode()
            self.b += struct.pack("<I", len(e)) + e + b"\0"
        elif c == "g":
            e = v.encode()
            self.b += bytes([len(e)]) + e + b"\0"
        elif c == "v":
            sig, inner = v
            self.put("g", sig)
            self.put(sig, inner)
        elif c == "a":
            self.pad(4)
            at = len(self.b)
            self.b += b"\0\0\0\0"
            self.pad(_ALIGN[t[1]])
            start = len(self.b)
            for x in v:
                self.put(t[1:], x)
            struct.pack_into("<I", self.b, at, len(self.b) - start)
        elif c in "({":
            self.pad(8)
            for st, x in zip(_split(t[1:-1]), v):
                self.put(st, x)
        else:
            raise ValueError(t)


class R:
    def __init__(self, b: bytes, p: int = 0):
        self.b, self.p = b, p

    def pad(self, n):
        self.p = (self.p + n - 1) // n * n

    def get(self, t: str):
        c = t[0]
        if c == "y":
            self.p += 1
            return self.b[self.p - 1]
        if c in "bu":
            self.pad(4)
            v = struct.unpack_from("<I", self.b, self.p)[0]
            self.p += 4
            return bool(v) if c == "b" else v
        if c == "i":
            self.pad(4)
            v = struct.unpack_from("<i", self.b, self.p)[0]
            self.p += 4
            return v
        if c in "so":
            self.pad(4)
            n = struct.unpack_from("<I", self.b, self.p)[0]
            s = self.b[self.p + 4:self.p + 4 + n].decode()
            self.p += 4 + n + 1
            return s
        if c == "g":
            n = self.b[self.p]
            s = self.b[self.p + 1:self.p + 1 + n].decode()
            self.p += n + 2
            return s
        if c == "v":
            sig = self.get("g")
            return (sig, self.get(sig))
        if c == "a":
            self.pad(4)
            n = struct.unpack_from("<I", self.b, self.p)[0]
            self.p += 4
            self.pad(_ALIGN[t[1]])
            end = self.p + n
            out = []
            while self.p < end:
                out.append(self.get(t[1:]))
            return out
        if c in "({":
            self.pad(8)
            return [self.get(st) for st in _split(t[1:-1])]
        raise ValueError(t)


FIELDS = {1: ("path", "o"), 2: ("interface", "s"), 3: ("member", "s"), 4: ("error_name", "s"), 5: ("reply_serial", "u"),
          6: ("destination", "s"), 7: ("sender", "s"), 8: ("signature", "g")}


def encode(msg_type: int, serial: int, fields: Dict[str, object], body_sig: str = "", body: Tuple = ()) -> bytes:
    bw = W()
    for t, v in zip(_split(body_sig), body):
        bw.put(t, v)
    hdr = W()
    hdr.b += b"l" + bytes([msg_type, 0, 1]) + struct.pack("<II", len(bw.b), serial)
    arr = []
    if body_sig:
        fields = dict(fields, signature=body_sig)
    for code, (name, sig) in FIELDS.items():
        if name in fields and fields[name] not in (None, ""):
            arr.append([code, (sig, fields[name])])
    hdr.put("a(yv)", arr)
    hdr.pad(8)
    return bytes(hdr.b + bw.b)


def decode(buf: bytes):
    """Returns (message dict, bytes consumed) or (None, 0) if incomplete."""
    if len(buf) < 16:
        return None, 0
    body_len, serial, flen = struct.unpack_from("<III", buf, 4)
    hdr_end = 16 + flen
    body_start = (hdr_end + 7) // 8 * 8
    total = body_start + body_len
    if len(buf) < total:
        return None, 0
    r = R(buf[:hdr_end], 12)
    fields = {}
    for code, (sig, val) in r.get("a(yv)"):
        if code in FIELDS:
            fields[FIELDS[code][0]] = val
    body = []
    if fields.get("signature"):
        br = R(buf[body_start:total])
        body = [br.get(t) for t in _split(fields["signature"])]
    return {"type": buf[1], "serial": serial, **fields, "body": body}, total


# ---------------------------------------------------------------------------
# server
# ---------------------------------------------------------------------------
class NetworkManagerModel:
    """The NetworkManager subset the agent uses (Version, GetAllDevices, Device.Interface and
    Device.Managed), answering decoded method calls with encoded replies."""

    NM = "org.freedesktop.NetworkManager"
    NM_PATH = "/org/freedesktop/NetworkManager"
    DEV_IFACE = "org.freedesktop.NetworkManager.Device"

    def __init__(self, devices: Dict[str, bool], nm_running: bool = True, fail_set: bool = False):
        self.devices = dict(devices)  # ifname -> Managed
        self.nm_running = nm_running
        self.fail_set = fail_set
        self.calls: List[Tuple[str, str, str]] = []
        self.auth_lines: List[str] = []

    def _err(self, m, serial, name, text):
        # Through a real bus a reply must be addressed to the caller's unique name.
        return encode(3, serial, {"reply_serial": m["serial"], "error_name": name, "destination": m.get("sender")},
                      "s", (text,))

    def _handle(self, m, serial) -> bytes:
        self.calls.append((m.get("path", ""), m.get("interface", ""), m.get("member", "")))
        ret = lambda sig="", body=(): encode(2, serial, {"reply_serial": m["serial"],  # noqa: E731
                                                         "destination": m.get("sender")}, sig, body)
        member, iface, path = m.get("member"), m.get("interface"), m.get("path", "")
        if iface == "org.freedesktop.DBus" and member == "Hello":
            return ret("s", (":1.42",))
        if m.get("destination") == self.NM and not self.nm_running:
            return self._err(m, serial, "org.freedesktop.DBus.Error.ServiceUnknown",
                             "The name org.freedesktop.NetworkManager was not provided by any .service files")
        names = sorted(self.devices)
        if iface == self.NM and member == "GetAllDevices":
            return ret("ao", ([f"{self.NM_PATH}/Devices/{i + 1}" for i in range(len(names))],))
        if iface == "org.freedesktop.DBus.Properties" and member == "Get":
            want_iface, prop = m["body"]
            if path == self.NM_PATH and prop == "Version":
                return ret("v", (("s", "1.46.0"),))
            if path.startswith(self.NM_PATH + "/Devices/") and prop == "Interface":
                return ret("v", (("s", names[int(path.rsplit("/", 1)[1]) - 1]),))
            if path.startswith(self.NM_PATH + "/Devices/") and prop == "Managed":
                return ret("v", (("b", self.devices[names[int(path.rsplit("/", 1)[1]) - 1]]),))
        if iface == "org.freedesktop.DBus.Properties" and member == "Set":
            _, prop, (sig, val) = m["body"]
            if prop == "Managed" and path.startswith(self.NM_PATH + "/Devices/"):
                if self.fail_set:
                    return self._err(m, serial, "org.freedesktop.NetworkManager.PermissionDenied", "not authorized")
                self.devices[names[int(path.rsplit("/", 1)[1]) - 1]] = bool(val)
                return ret()
        return self._err(m, serial, "org.freedesktop.DBus.Error.UnknownMethod", f"no method {iface}.{member}")


class FakeNetworkManagerBus(NetworkManagerModel):
    """Serves one or more clients on a UNIX socket until ``stop``, as if it were the bus."""

    def __init__(self, path: str, devices: Dict[str, bool], nm_running: bool = True, fail_set: bool = False):
        super().__init__(devices, nm_running, fail_set)
        self.path = path
        self._sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        if os.path.exists(path):
            os.unlink(path)
        self._sock.bind(path)
        self._sock.listen(4)
        self._stop = False
        self._threads: List[threading.Thread] = []
        t = threading.Thread(target=self._accept, daemon=True)
        t.start()
        self._threads.append(t)

    @property
    def address(self) -> str:
        return f"unix:path={self.path}"

    def stop(self):
        self._stop = True
        try:
            self._sock.close()
        except OSError:
            pass

    def _accept(self):
        while not self._stop:
            try:
                c, _ = self._sock.accept()
            except OSError:
                return
            t = threading.Thread(target=self._serve, args=(c,), daemon=True)
            t.start()
            self._threads.append(t)

    def _serve(self, c: socket.socket):
        buf = b""
        try:
            # SASL: a NUL byte then CRLF-terminated lines until BEGIN
            while b"BEGIN\r\n" not in buf:
                d = c.recv(4096)
                if not d:
                    return
                buf += d
                while b"\r\n" in buf and not buf.startswith(b"BEGIN"):
                    line, buf = buf.split(b"\r\n", 1)
                    line = line.lstrip(b"\0").decode()
                    self.auth_lines.append(line)
                    if line.startswith("AUTH EXTERNAL "):
                        uid = bytes.fromhex(line.split()[2]).decode()
                        ok = uid == str(os.getuid())
                        c.sendall(b"OK 0123456789abcdef0123456789abcdef\r\n" if ok else b"REJECTED EXTERNAL\r\n")
                    elif line.startswith("AUTH"):
                        c.sendall(b"REJECTED EXTERNAL\r\n")
            buf = buf.split(b"BEGIN\r\n", 1)[1]
            serial = 1000
            while True:
                m, used = decode(buf)
                if m is None:
                    d = c.recv(65536)
                    if not d:
                        return
                    buf += d
                    continue
                buf = buf[used:]
                serial += 1
                c.sendall(self._handle(m, serial))
        except OSError:
            return
        finally:
            c.close()


class NetworkManagerOnBus(NetworkManagerModel):
    """Owns ``org.freedesktop.NetworkManager`` on a real bus (a client of ``dbus-daemon``) and
    answers the same calls as ``FakeNetworkManagerBus``."""

    def __init__(self, address: str, devices: Dict[str, bool], fail_set: bool = False):
        super().__init__(devices, nm_running=True, fail_set=fail_set)
        self._stop = False
        path = address.split("unix:path=", 1)[1].split(",", 1)[0]
        self._c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self._c.connect(path)
        self._c.sendall(b"\0AUTH EXTERNAL " + str(os.getuid()).encode().hex().encode() + b"\r\n")
        line = self._line()
        if not line.startswith("OK "):
            raise RuntimeError(f"dbus-daemon refused the service: {line}")
        self._c.sendall(b"BEGIN\r\n")
        self._buf = b""
        self._serial = 0
        self.unique_name = self._call("org.freedesktop.DBus", "/org/freedesktop/DBus", "org.freedesktop.DBus", "Hello")[0]
        # flags 4 = DBUS_NAME_FLAG_DO_NOT_QUEUE; reply 1 = PRIMARY_OWNER
        owner = self._call("org.freedesktop.DBus", "/org/freedesktop/DBus", "org.freedesktop.DBus", "RequestName",
                           "su", (self.NM, 4))[0]
        if owner != 1:
            raise RuntimeError(f"could not own {self.NM}: RequestName -> {owner}")
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()

    def _line(self) -> str:
        b = b""
        while not b.endswith(b"\r\n"):
            d = self._c.recv(1)
            if not d:
                raise RuntimeError("bus closed during authentication")
            b += d
        return b[:-2].decode()

    def _read(self):
        while True:
            m, used = decode(self._buf)
            if m is not None:
                self._buf = self._buf[used:]
                return m
            d = self._c.recv(65536)
            if not d:
                return None
            self._buf += d

    def _call(self, dest, path, iface, member, sig="", body=()):
        self._serial += 1
        self._c.sendall(encode(1, self._serial, {"path": path, "interface": iface, "member": member,
                                                 "destination": dest}, sig, body))
        while True:
            m = self._read()
            if m is None:
                raise RuntimeError("bus closed")
            if m["type"] in (2, 3) and m.get("reply_serial") == self._serial:
                if m["type"] == 3:
                    raise RuntimeError(f"{m.get('error_name')}: {m['body']}")
                return m["body"]

    def _loop(self):
        serial = 5000
        try:
            while not self._stop:
                m = self._read()
                if m is None:
                    return
                if m["type"] != 1:  # signals (NameAcquired, ...) and stray replies
                    continue
                serial += 1
                self._c.sendall(self._handle(m, serial))
        except OSError:
            return

    def stop(self):
        self._stop = True
        try:
            self._c.shutdown(socket.SHUT_RDWR)
            self._c.close()
        except OSError:
            pass


class BusDaemon:
    """A private ``dbus-daemon`` (freedesktop's reference bus) on a UNIX socket under ``tmpdir``."""

    CONFIG = """<!DOCTYPE busconfig PUBLIC "-//freedesktop//DTD D-Bus Bus Configuration 1.0//EN"
 "http://www.freedesktop.org/standards/dbus/1.0/busconfig.dtd">
<busconfig>
  <type>system</type>
  <listen>unix:path={path}</listen>
  <auth>EXTERNAL</auth>
  <policy context="default">
    <allow user="*"/>
    <allow own="*"/>
    <allow send_type="method_call"/>
    <allow receive_type="method_call"/>
    <allow send_destination="*"/>
    <allow receive_type="method_return"/>
    <allow receive_type="error"/>
    <allow receive_type="signal"/>
  </policy>
</busconfig>
"""

    @staticmethod
    def available() -> Optional[str]:
        return shutil.which("dbus-daemon")

    def __init__(self, tmpdir: str):
        exe = self.available()
        if not exe:
            raise FileNotFoundError("dbus-daemon not installed")
        d = Path(tmpdir)
        self.socket_path = str(d / "system_bus_socket")
        conf = d / "bus.conf"
        conf.write_text(self.CONFIG.format(path=self.socket_path))
        self.proc = subprocess.Popen([exe, f"--config-file={conf}", "--nofork", "--nopidfile", "--print-address"],
                                     stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        line = self.proc.stdout.readline().strip()
        if not line.startswith("unix:"):
            err = self.proc.stderr.read() if self.proc.poll() is not None else ""
            self.stop()
            raise RuntimeError(f"dbus-daemon did not start: {line!r} {err}")
        self.address = line

    def stop(self):
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
