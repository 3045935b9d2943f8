"""Kernel resource metadata of the built library's gfx950 code objects (test infrastructure).

`libocvf_hip.so` carries one clang offload bundle per translation unit, concatenated in its
`.hip_fatbin` section.  `kernel_resources()` splits the bundles, takes each gfx950 code object and
reads the AMDGPU metadata note (`llvm-readelf --notes`): per kernel symbol the VGPR/AGPR/SGPR
counts, the spill counts and the private (scratch) segment size.  `disassemble()` gives the ISA
of one kernel for hazard checks.  Host-only: nothing here touches a GPU.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FIELDS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "private_segment_fixed_size")


def code_objects(lib_path: str) -> list[bytes]:
    """Every gfx950 code object of the library's offload bundles."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib_path,
                        os.path.join(td, "discard.so")], check=True, capture_output=True)
        data = open(fat, "rb").read()
    out = []
    for m in re.finditer(re.escape(MAGIC), data):
        p = m.start()
        (ne,) = struct.unpack_from("<Q", data, p + 24)
        o = p + 32
        for _ in range(ne):
            off, size, tl = struct.unpack_from("<QQQ", data, o)
            o += 24
            triple = data[o:o + tl].decode()
            o += tl
            if "gfx950" in triple:
                out.append(data[p + off:p + off + size])
    return out


def _notes(elf: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(elf)
        f.flush()
        return subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], check=True,
                              capture_output=True, text=True).stdout


def kernel_resources(lib_path: str) -> dict[str, dict[str, int]]:
    """{kernel symbol (mangled): {field: value}} over all code objects of the library."""
    res: dict[str, dict[str, int]] = {}
    for elf in code_objects(lib_path):
        cur: dict[str, int] = {}
        name = None
        # the metadata lists each kernel's keys in alphabetical order (.agpr_count first, the vgpr
        # fields after .symbol): a kernel's entry ends where the next one's .agpr_count starts
        for line in _notes(elf).splitlines() + ["- .agpr_count: 0"]:
            s = line.strip()
            if s.startswith("- .agpr_count:"):
                if name is not None:
                    res[name] = cur
                cur, name = {}, None
            m = re.match(r"-?\s*\.(\w+):\s+(.*)$", s)
            if not m:
                continue
            k, v = m.group(1), m.group(2).strip()
            if k in FIELDS:
                cur[k] = int(v)
            elif k == "symbol":
                name = v[:-3] if v.endswith(".kd") else v
    return res


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True, check=True).stdout.splitlines()
    return dict(zip(names, out))


def disassemble(lib_path: str, symbol: str) -> list[str]:
    """The ISA lines of one kernel (mangled symbol)."""
    for elf in code_objects(lib_path):
        with tempfile.NamedTemporaryFile(suffix=".elf") as f:
            f.write(elf)
            f.flush()
            syms = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-s", f.name], capture_output=True,
                                  text=True, check=True).stdout
            if f" {symbol}\n" not in syms + "\n" and not re.search(rf"\s{re.escape(symbol)}$", syms, re.M):
                continue
            txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn",
                                  f"--disassemble-symbols={symbol}", f.name], capture_output=True, text=True,
                                 check=True).stdout
            return [ln.strip() for ln in txt.splitlines() if ln.startswith("\t") or ln.startswith(" ")]
    raise KeyError(symbol)
