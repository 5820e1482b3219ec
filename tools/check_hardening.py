#!/usr/bin/env python3
"""Binary-hardening gate for the agent image (the reference's checksec step,
reference build/Dockerfile.linkdiscovery:36-41), as a dependency-free ELF reader.

The reference runs checksec on its binaries. Neither checksec nor a network to fetch it exists
here, and the image build should not need binutils. So the ELF is read directly:

* PIE: ``e_type == ET_DYN`` with a ``PT_INTERP`` segment (an executable, not a plain shared
  object), or ``DF_1_PIE``;
* full RELRO: a ``PT_GNU_RELRO`` segment plus immediate binding (``DF_BIND_NOW`` or ``DF_1_NOW``);
* non-executable stack: ``PT_GNU_STACK`` without ``PF_X``;
* stack protector: an undefined ``__stack_chk_fail`` in the dynamic symbols;
* FORTIFY_SOURCE: at least one ``__*_chk`` import.

Usage: ``check_hardening.py BINARY...``. It prints one line per binary and exits 1 if any check
fails. ``tests/test_hardening.py`` runs it on the built binaries, and the agent image's builder
stage runs it before the runtime stage copies them.
"""

from __future__ import annotations

import json
import struct
import sys
from typing import Dict, List

ET_DYN = 3
PT_DYNAMIC, PT_INTERP = 2, 3
PT_GNU_STACK, PT_GNU_RELRO = 0x6474E551, 0x6474E552
PF_X = 1
DT_NULL, DT_FLAGS, DT_FLAGS_1 = 0, 30, 0x6FFFFFFB
DF_BIND_NOW = 0x8
DF_1_NOW, DF_1_PIE = 0x1, 0x08000000
SHT_DYNSYM = 11


class ElfError(ValueError):
    pass


def _read(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


def inspect(path: str) -> Dict[str, object]:
    b = _read(path)
    if b[:4] != b"\x7fELF":
        raise ElfError(f"{path}: not an ELF file")
    if b[4] != 2 or b[5] != 1:
        raise ElfError(f"{path}: only 64-bit little-endian ELF is supported")
    (e_type, _mach, _ver, _entry, e_phoff, e_shoff, _flags, _ehsize, e_phentsize, e_phnum, e_shentsize, e_shnum,
     _shstrndx) = struct.unpack_from("<HHIQQQIHHHHHH", b, 16)
    phdrs = [struct.unpack_from("<IIQQQQQQ", b, e_phoff + i * e_phentsize) for i in range(e_phnum)]
    types = {p[0] for p in phdrs}
    stack = [p for p in phdrs if p[0] == PT_GNU_STACK]
    flags = flags_1 = 0
    for p in phdrs:
        if p[0] != PT_DYNAMIC:
            continue
        off, size = p[2], p[5]
        for i in range(size // 16):
            tag, val = struct.unpack_from("<qQ", b, off + 16 * i)
            if tag == DT_NULL:
                break
            if tag == DT_FLAGS:
                flags = val
            elif tag == DT_FLAGS_1:
                flags_1 = val
    imports: List[str] = []
    shdrs = [struct.unpack_from("<IIQQQQIIQQ", b, e_shoff + i * e_shentsize) for i in range(e_shnum)] if e_shoff else []
    for sh in shdrs:
        if sh[1] != SHT_DYNSYM:
            continue
        str_sh = shdrs[sh[6]]
        stroff = str_sh[4]
        entsize = sh[9] or 24
        for i in range(sh[5] // entsize):
            st_name, _info, _other, st_shndx, _value, _size = struct.unpack_from("<IBBHQQ", b, sh[4] + i * entsize)
            if st_shndx != 0 or not st_name:
                continue  # defined here, or the null symbol
            end = b.index(b"\0", stroff + st_name)
            imports.append(b[stroff + st_name:end].decode(errors="replace"))
    fortified = sorted(s for s in imports if s.startswith("__") and s.endswith("_chk") and s != "__stack_chk_fail")
    return {
        "path": path,
        "pie": e_type == ET_DYN and (PT_INTERP in types or bool(flags_1 & DF_1_PIE)),
        "relro": PT_GNU_RELRO in types,
        "bind_now": bool(flags & DF_BIND_NOW) or bool(flags_1 & DF_1_NOW),
        "nx_stack": bool(stack) and not (stack[0][1] & PF_X),
        "stack_protector": "__stack_chk_fail" in imports,
        "fortify": fortified,
    }


CHECKS = ("pie", "relro", "bind_now", "nx_stack", "stack_protector", "fortify")


def failures(report: Dict[str, object]) -> List[str]:
    return [c for c in CHECKS if not report[c]]


def main(argv=None) -> int:
    paths = list(sys.argv[1:] if argv is None else argv)
    if not paths:
        print(__doc__, file=sys.stderr)
        return 2
    bad = 0
    for p in paths:
        try:
            r = inspect(p)
        except (OSError, ElfError, struct.error) as e:
            print(f"FAIL {p}: {e}")
            bad += 1
            continue
        f = failures(r)
        bad += bool(f)
        print(("FAIL " if f else "ok   ") + json.dumps(dict(r, fortify=len(r["fortify"]), missing=f)))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
