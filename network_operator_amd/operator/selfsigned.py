"""Self-signed serving certificates generated in process: ECDSA P-256 keys, X.509 v3 DER, PEM.

controller-runtime self-signs in memory when ``--metrics-secure`` has no certificate to load
(reference cmd/operator/main.go:157-167, through its ``certwatcher`` fallback).  The operator
image is distroless (no ``openssl`` binary) and carries no crypto package beyond the ``ssl``
module, which can load a certificate but not make one.  So the key pair, the signature and the
DER encoding are done here, in a few hundred lines of plain Python: NIST P-256 arithmetic in
Jacobian coordinates, ECDSA with SHA-256 (RFC 6979 deterministic nonces, so no weak random ``k``
can leak the key), and the ASN.1 DER of one certificate shape:

* version 3, a random positive 127-bit serial, issuer = subject = ``CN=<cn>``;
* ``subjectAltName`` (DNS names and IPv4/IPv6 addresses) and ``basicConstraints CA:TRUE``, so a
  client can trust the certificate itself as its CA (the caBundle of a webhook configuration);
* ``keyUsage`` digitalSignature + keyCertSign, ``subjectKeyIdentifier``.

Written by this module only for the serving endpoints; it is no general X.509 library.
"""

from __future__ import annotations

import datetime as _dt
import hashlib
import hmac
import ipaddress
import secrets
from pathlib import Path
from typing import Iterable, Optional, Tuple

# --- NIST P-256 (SEC 2, section 2.4.2) --------------------------------------------------------
P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
A = P - 3
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5
G = (GX, GY)


def _jdouble(x, y, z):
    if not y:
        return (0, 1, 0)
    ysq = y * y % P
    s = 4 * x * ysq % P
    zsq = z * z % P
    m = 3 * (x - zsq) * (x + zsq) % P  # a = -3
    nx = (m * m - 2 * s) % P
    ny = (m * (s - nx) - 8 * ysq * ysq) % P
    nz = 2 * y * z % P
    return (nx, ny, nz)


def _jadd(p1, p2):
    x1, y1, z1 = p1
    x2, y2, z2 = p2
    if not z1:
        return p2
    if not z2:
        return p1
    z1s, z2s = z1 * z1 % P, z2 * z2 % P
    u1, u2 = x1 * z2s % P, x2 * z1s % P
    s1, s2 = y1 * z2s * z2 % P, y2 * z1s * z1 % P
    if u1 == u2:
        return _jdouble(x1, y1, z1) if s1 == s2 else (0, 1, 0)
    h, r = (u2 - u1) % P, (s2 - s1) % P
    h2 = h * h % P
    h3 = h * h2 % P
    u1h2 = u1 * h2 % P
    nx = (r * r - h3 - 2 * u1h2) % P
    ny = (r * (u1h2 - nx) - s1 * h3) % P
    nz = h * z1 * z2 % P
    return (nx, ny, nz)


def scalar_mult(k: int, point: Tuple[int, int] = G) -> Tuple[int, int]:
    """k * point in affine coordinates (the point at infinity is not returned for 0 < k < N)."""
    acc = (0, 1, 0)
    add = (point[0], point[1], 1)
    for bit in bin(k)[2:]:
        acc = _jdouble(*acc)
        if bit == "1":
            acc = _jadd(acc, add)
    x, y, z = acc
    if not z:
        raise ValueError("point at infinity")
    zi = pow(z, -1, P)
    zi2 = zi * zi % P
    return (x * zi2 % P, y * zi2 * zi % P)


def on_curve(pt: Tuple[int, int]) -> bool:
    x, y = pt
    return (y * y - (x * x * x + A * x + B)) % P == 0


def _rfc6979_k(d: int, h: bytes):
    """Deterministic nonces for (key d, message hash h) (RFC 6979 section 3.2, HMAC-SHA256)."""
    x = d.to_bytes(32, "big")
    h1 = (int.from_bytes(h, "big") % N).to_bytes(32, "big")
    v, k = b"\x01" * 32, b"\x00" * 32
    k = hmac.new(k, v + b"\x00" + x + h1, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    k = hmac.new(k, v + b"\x01" + x + h1, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    while True:
        v = hmac.new(k, v, hashlib.sha256).digest()
        cand = int.from_bytes(v, "big")
        if 1 <= cand < N:
            yield cand
        k = hmac.new(k, v + b"\x00", hashlib.sha256).digest()
        v = hmac.new(k, v, hashlib.sha256).digest()


def sign(d: int, message: bytes) -> Tuple[int, int]:
    """ECDSA-SHA256 signature (r, s) of `message` with private scalar d (low-s form)."""
    h = hashlib.sha256(message).digest()
    e = int.from_bytes(h, "big")
    for k in _rfc6979_k(d, h):
        r = scalar_mult(k)[0] % N
        if not r:
            continue
        s = pow(k, -1, N) * (e + r * d) % N
        if not s:
            continue
        return r, min(s, N - s)
    raise AssertionError("unreachable")


def verify(q: Tuple[int, int], message: bytes, sig: Tuple[int, int]) -> bool:
    r, s = sig
    if not (1 <= r < N and 1 <= s < N) or not on_curve(q):
        return False
    e = int.from_bytes(hashlib.sha256(message).digest(), "big")
    w = pow(s, -1, N)
    u1, u2 = e * w % N, r * w % N
    p1 = (*scalar_mult(u1), 1)
    p2 = (*scalar_mult(u2, q), 1)
    x, _, z = _jadd(p1, p2)
    if not z:
        return False
    zi = pow(z, -1, P)
    return x * zi * zi % P % N == r


# --- ASN.1 DER --------------------------------------------------------------------------------
def _len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _tlv(tag: int, body: bytes) -> bytes:
    return bytes([tag]) + _len(len(body)) + body


def der_int(v: int) -> bytes:
    b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")  # a leading 0 keeps it positive
    return _tlv(0x02, b)


def der_seq(*items: bytes) -> bytes:
    return _tlv(0x30, b"".join(items))


def der_set(*items: bytes) -> bytes:
    return _tlv(0x31, b"".join(items))


def der_oid(dotted: str) -> bytes:
    parts = [int(x) for x in dotted.split(".")]
    out = bytearray([40 * parts[0] + parts[1]])
    for p in parts[2:]:
        chunk = [p & 0x7F]
        p >>= 7
        while p:
            chunk.append(0x80 | (p & 0x7F))
            p >>= 7
        out += bytes(reversed(chunk))
    return _tlv(0x06, bytes(out))


def der_bitstring(b: bytes) -> bytes:
    return _tlv(0x03, b"\x00" + b)


def der_octets(b: bytes) -> bytes:
    return _tlv(0x04, b)


def der_utf8(s: str) -> bytes:
    return _tlv(0x0C, s.encode())


def der_bool(v: bool) -> bytes:
    return _tlv(0x01, b"\xff" if v else b"\x00")


def der_time(t: _dt.datetime) -> bytes:
    t = t.astimezone(_dt.timezone.utc)
    if 1950 <= t.year < 2050:
        return _tlv(0x17, t.strftime("%y%m%d%H%M%SZ").encode())  # UTCTime
    return _tlv(0x18, t.strftime("%Y%m%d%H%M%SZ").encode())  # GeneralizedTime


def _explicit(n: int, body: bytes) -> bytes:
    return _tlv(0xA0 | n, body)


OID_EC_PUBLIC_KEY = "1.2.840.10045.2.1"
OID_P256 = "1.2.840.10045.3.1.7"
OID_ECDSA_SHA256 = "1.2.840.10045.4.3.2"
OID_CN = "2.5.4.3"
OID_SAN = "2.5.29.17"
OID_BASIC_CONSTRAINTS = "2.5.29.19"
OID_KEY_USAGE = "2.5.29.15"
OID_SKI = "2.5.29.14"


def pem(label: str, der: bytes) -> str:
    import base64

    b64 = base64.b64encode(der).decode()
    lines = [b64[i:i + 64] for i in range(0, len(b64), 64)]
    return f"-----BEGIN {label}-----\n" + "\n".join(lines) + f"\n-----END {label}-----\n"


def _san(names: Iterable[str]) -> bytes:
    """subjectAltName entries "DNS:host" / "IP:addr" (the openssl -addext spelling)."""
    out = b""
    for n in names:
        kind, _, value = n.partition(":")
        if kind == "DNS":
            out += _tlv(0x82, value.encode())  # [2] IMPLICIT IA5String
        elif kind == "IP":
            out += _tlv(0x87, ipaddress.ip_address(value).packed)  # [7] IMPLICIT OCTET STRING
        else:
            raise ValueError(f"unsupported subjectAltName {n!r}")
    return der_seq(out)


def make_certificate(cn: str = "localhost", sans: Iterable[str] = ("DNS:localhost", "IP:127.0.0.1"),
                     days: int = 365, now: Optional[_dt.datetime] = None,
                     key: Optional[int] = None) -> Tuple[bytes, bytes]:
    """(certificate DER, private key DER in SEC 1 form) of a new self-signed P-256 certificate."""
    d = key if key is not None else secrets.randbelow(N - 1) + 1
    qx, qy = scalar_mult(d)
    pub = b"\x04" + qx.to_bytes(32, "big") + qy.to_bytes(32, "big")
    now = now or _dt.datetime.now(_dt.timezone.utc)
    name = der_seq(der_set(der_seq(der_oid(OID_CN), der_utf8(cn))))
    algo = der_seq(der_oid(OID_ECDSA_SHA256))
    spki = der_seq(der_seq(der_oid(OID_EC_PUBLIC_KEY), der_oid(OID_P256)), der_bitstring(pub))
    ski = hashlib.sha1(pub).digest()
    exts = der_seq(
        der_seq(der_oid(OID_SAN), der_octets(_san(sans))),
        der_seq(der_oid(OID_BASIC_CONSTRAINTS), der_bool(True), der_octets(der_seq(der_bool(True)))),
        # keyUsage: digitalSignature (bit 0) + keyCertSign (bit 5): 0b10000100, 2 unused bits
        der_seq(der_oid(OID_KEY_USAGE), der_bool(True), der_octets(_tlv(0x03, b"\x02\x84"))),
        der_seq(der_oid(OID_SKI), der_octets(der_octets(ski))),
    )
    tbs = der_seq(
        _explicit(0, der_int(2)),
        der_int(secrets.randbits(127) | 1),
        algo,
        name,
        der_seq(der_time(now - _dt.timedelta(minutes=5)), der_time(now + _dt.timedelta(days=days))),
        name,
        spki,
        _explicit(3, exts),
    )
    r, s = sign(d, tbs)
    cert = der_seq(tbs, algo, der_bitstring(der_seq(der_int(r), der_int(s))))
    sec1 = der_seq(der_int(1), der_octets(d.to_bytes(32, "big")), _explicit(0, der_oid(OID_P256)),
                   _explicit(1, der_bitstring(pub)))
    return cert, sec1


def write_self_signed(cert_dir: Path, cn: str = "localhost", sans: Iterable[str] = ("DNS:localhost", "IP:127.0.0.1"),
                      days: int = 365) -> Tuple[Path, Path]:
    """tls.crt / tls.key (PEM) in `cert_dir`; the key is written 0600 before it has content."""
    import os

    cert_dir = Path(cert_dir)
    cert_dir.mkdir(parents=True, exist_ok=True)
    der, key = make_certificate(cn, sans, days)
    crt_path, key_path = cert_dir / "tls.crt", cert_dir / "tls.key"
    fd = os.open(key_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    os.fchmod(fd, 0o600)  # a key file that already existed keeps its mode through O_CREAT
    with os.fdopen(fd, "w") as f:
        f.write(pem("EC PRIVATE KEY", key))
    crt_path.write_text(pem("CERTIFICATE", der))
    return crt_path, key_path
