"""Spill guard of the inline-asm MFMA kernels (CPU: reads the built library's gfx950 code objects).

The hot engines issue their MFMAs as inline asm (accumulators pinned in AGPRs / VGPRs), and the
compiler's hazard recognizer does not see into asm: a spill store placed behind such an MFMA before
its result is written stores a stale accumulator, a scratch load into a register an executing MFMA
still reads corrupts its operand.  DESIGN.md §3 ("Precision design") records both failure modes from
rounds 3 and 5.  So:

* the kernels in ZERO must have no VGPR or SGPR spills and no scratch segment at all;
* every other asm-MFMA kernel (ALLOWED, with the counts it is known to carry) may keep spills of
  loop invariants, but no scratch instruction may sit within the hazard window of an MFMA: between two
  MFMAs of one block, or fewer than HAZARD wait states after the last MFMA of a block in program order.
"""
from __future__ import annotations

import os
import re
import sys

import pytest

sys.path.insert(0, os.path.dirname(__file__))
import _codeobj as C  # noqa: E402

LIB = os.path.join(os.path.dirname(__file__), "..", "opencv_facerecognizer_amd", "libocvf_hip.so")

# demangled-name prefixes
ZERO = [
    "void ofr::q8::project_q8w_kernel<false>(",
    "void ofr::q8::project_q8w_kernel<true>(",
    "void ofr::q8s::tile_kernel_f6w<1>(",
]
# asm-MFMA kernels allowed to keep invariant spills, with upper bounds on the counts
ALLOWED = {
    "void ofr::q8s::tile_kernel_f6p<1>(": dict(vgpr_spill_count=8, sgpr_spill_count=8),
    "void ofr::q8s::tile_kernel_f6p<2>(": dict(vgpr_spill_count=8, sgpr_spill_count=8),
    "void ofr::q8s::tile_kernel_f6w<3>(": dict(vgpr_spill_count=24, sgpr_spill_count=8),
    "void ofr::q8s::tile_kernel<2>(": dict(vgpr_spill_count=8, sgpr_spill_count=48),
}
# builtin-MFMA kernels (the compiler sees their hazards) held to no VGPR spills and no scratch: their SGPR
# spills go to VGPR lanes (v_writelane), not memory.  The round-6 folded prefix pass spilled 531 VGPRs of
# hoisted hit payloads until its lane index was laundered per column block.
NO_SCRATCH = [
    "void ofr::q8s::prefix_wave_kernel<4, 4, 1>(",
    "void ofr::q8s::prefix_wave_kernel<4, 4, 2>(",
    "void ofr::q8s::prefix_wave_kernel<8, 2, 1>(",
    "ofr::q8s::sample_wave_kernel(",
    "void ofr::q8s::prefix_pass_kernel<true>(",
    "void ofr::q8s::prefix_pass_kernel<false>(",
]
# wait states an XDL result needs before any reader (16-pass MFMA: 18 on gfx950) plus margin
HAZARD = 24

pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libocvf_hip.so not built")


@pytest.fixture(scope="module")
def resources():
    r = C.kernel_resources(LIB)
    dm = C.demangle(list(r))
    return {dm[k]: (k, v) for k, v in r.items()}


def _find(resources, prefix):
    hits = [(n, kv) for n, kv in resources.items() if n.startswith(prefix)]
    assert len(hits) == 1, (prefix, [n for n, _ in hits])
    return hits[0][1]


@pytest.mark.parametrize("prefix", ZERO)
def test_no_spills_no_scratch(resources, prefix):
    _, v = _find(resources, prefix)
    assert v.get("vgpr_spill_count", 0) == 0, (prefix, v)
    assert v.get("sgpr_spill_count", 0) == 0, (prefix, v)
    assert v.get("private_segment_fixed_size", 0) == 0, (prefix, v)


def _wait_states(line: str) -> int:
    m = re.match(r"s_nop\s+(\d+)", line)
    return int(m.group(1)) + 1 if m else 1


def scratch_in_hazard_window(lines: list[str]) -> list[str]:
    """Scratch instructions inside an MFMA block or within HAZARD wait states after one."""
    bad = []
    mf = [i for i, ln in enumerate(lines) if ln.startswith("v_mfma")]
    for i, ln in enumerate(lines):
        if not ln.startswith("scratch_"):
            continue
        prev = [j for j in mf if j < i]
        nxt = [j for j in mf if j > i]
        if not prev:
            continue
        p = prev[-1]
        ws = sum(_wait_states(lines[k]) for k in range(p + 1, i))
        # an MFMA follows closely without a barrier in between: the scratch op sits inside a block
        inside = bool(nxt) and nxt[0] - i < 32 and not any("s_barrier" in lines[k] for k in range(i, nxt[0]))
        if ws < HAZARD or (inside and ws < 4 * HAZARD):
            bad.append(f"{i}: {ln} ({ws} wait states after MFMA at {p})")
    return bad


@pytest.mark.parametrize("prefix", NO_SCRATCH)
def test_no_vgpr_spills_no_scratch(resources, prefix):
    _, v = _find(resources, prefix)
    assert v.get("vgpr_spill_count", 0) == 0, (prefix, v)
    assert v.get("private_segment_fixed_size", 0) == 0, (prefix, v)


@pytest.mark.parametrize("prefix", sorted(ALLOWED))
def test_allowed_spills_outside_mfma_hazards(resources, prefix):
    sym, v = _find(resources, prefix)
    for k, cap in ALLOWED[prefix].items():
        assert v.get(k, 0) <= cap, (prefix, k, v)
    lines = C.disassemble(LIB, sym)
    assert any(ln.startswith("v_mfma") for ln in lines), prefix
    bad = scratch_in_hazard_window(lines)
    assert not bad, (prefix, bad[:8])


def test_hazard_check_flags_a_spill_behind_an_mfma():
    lines = ["v_mfma_f32_16x16x32_f16 a[0:3], v[0:1], v[2:3], a[0:3]", "v_accvgpr_read_b32 v1, a0",
             "scratch_store_dword off, v1, off", "s_nop 7", "s_nop 7", "s_nop 7",
             "scratch_load_dword v2, off, off"]
    bad = scratch_in_hazard_window(lines)
    assert len(bad) == 1 and "scratch_store" in bad[0]
