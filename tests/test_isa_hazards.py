"""ISA audit of the inline-asm MFMA GEMM kernels (CPU: hipcc cross-compiles).

The GEMMs pin their accumulators to AGPRs with inline-asm MFMAs, which hipcc's
hazard recognizer cannot see.  A v_accvgpr_read/mov of an accumulator issued
within a few instructions of the asm MFMA that writes it reads a stale value
(two schedules produced wrong tiles this way: register-allocator copies at the
K-loop exit, ahead of the drain).  ``mxk::mfma_drain`` must sit between the last
MFMA and every accumulator read; this test scans the generated code for any
read of an AGPR within 12 instructions (an ``s_nop 7`` counts 8) of an MFMA
that wrote it.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _asm(src: str, out: str, flags: tuple = ()) -> str:
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", *flags,
                    "-I" + os.path.join(REPO, "native", "kernels"), "--cuda-device-only", "-S",
                    os.path.join(REPO, "native", "kernels", src), "-o", out],
                   check=True, capture_output=True)
    with open(out) as f:
        return f.read()


def close_accumulator_reads(asm: str) -> dict[str, int]:
    bad = {}
    for name in re.findall(r"^(_Z[^\s:]+):", asm, re.M):
        i = asm.find(name + ":")
        j = asm.find(".Lfunc_end", i)
        body = [ln.split(";")[0].strip() for ln in asm[i:j].split("\n")]
        body = [ln for ln in body if ln and not ln.startswith(".")]
        pend: dict[int, int] = {}
        n = 0
        for ln in body:
            if ln.startswith("v_mfma"):
                pend = {r: c + 1 for r, c in pend.items()}
                m = re.match(r"v_mfma\S*\s+a\[(\d+):(\d+)\]", ln)
                if m:
                    for r in range(int(m.group(1)), int(m.group(2)) + 1):
                        pend[r] = 0
                continue
            step = 8 if ln.startswith("s_nop 7") else 1
            pend = {r: c + step for r, c in pend.items() if c + step < 40}
            if ln.startswith(("v_accvgpr_read", "v_accvgpr_mov")):
                ops = ln.split(" ", 1)[1] if " " in ln else ""
                for m in re.finditer(r"\ba(\d+)\b", ops):
                    if int(m.group(1)) in pend and pend[int(m.group(1))] < 12:
                        n += 1
            elif ln.startswith(("scratch_store", "global_store", "buffer_store", "flat_store")):
                # a store straight from accumulators (e.g. a register-allocator
                # spill of an AGPR) reads them just like v_accvgpr_read
                ops = ln.split(" ", 1)[1] if " " in ln else ""
                for m in re.finditer(r"\ba\[(\d+):(\d+)\]|\ba(\d+)\b", ops):
                    lo = int(m.group(1) or m.group(3))
                    hi = int(m.group(2) or m.group(3))
                    if any(r in pend and pend[r] < 12 for r in range(lo, hi + 1)):
                        n += 1
        if n:
            bad[name] = n
    return bad


def _regs(text: str) -> set[int]:
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        lo = int(m.group(1) or m.group(3))
        hi = int(m.group(2) or m.group(3))
        out.update(range(lo, hi + 1))
    return out


def close_vgpr_result_reads(asm: str, states: int = 12) -> dict[str, int]:
    """Reads of an MFMA's VGPR result (``v_mfma ... v[a:b], ...``) by any
    instruction other than the next MFMA of its chain within ``states`` wait
    states (``s_nop N`` counts N + 1).  The 256-key attention backward keeps
    S / dP in VGPRs through inline-asm MFMAs, which hipcc does not pad: the
    VALU softmax must not read them early (8-pass XDL -> VALU: 12 states).
    Linear scan of the listing: fall-through only (an unconditional branch
    ends the tracking; jump targets are not followed)."""
    bad = {}
    for name in re.findall(r"^(_Z[^\s:]+):", asm, re.M):
        i = asm.find(name + ":")
        j = asm.find(".Lfunc_end", i)
        body = [ln.split(";")[0].strip() for ln in asm[i:j].split("\n")]
        body = [ln for ln in body if ln and not ln.startswith(".") and not ln.endswith(":")]
        pend: dict[int, int] = {}
        n = 0
        for ln in body:
            op, _, rest = ln.partition(" ")
            if op.startswith("v_mfma"):
                dst, _, srcs = rest.partition(",")
                # the chain's next MFMA may take the result whole as C
                pend = {r: c + 1 for r, c in pend.items() if r not in _regs(srcs.rsplit(",", 1)[0])
                        or c >= states}
                if dst.strip().startswith("v"):
                    for r in _regs(dst):
                        pend[r] = 0
                continue
            m = re.match(r"s_nop (\d+)", ln)
            step = int(m.group(1)) + 1 if m else 1
            if any(pend.get(r, states) < states for r in _regs(rest)):
                n += 1
            pend = {r: c + step for r, c in pend.items() if c + step < states}
            if op in ("s_branch", "s_endpgm", "s_setpc_b64"):
                pend = {}     # the next line is not reached by fall-through
        if n:
            bad[name] = n
    return bad


def test_detector_flags_a_close_vgpr_result_read():
    asm = ("_Zbaz:\n\tv_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]\n"
           "\tv_mfma_f32_32x32x16_bf16 v[0:15], v[24:27], v[28:31], v[0:15]\n"
           "\tv_mul_f32_e32 v40, 0x3fb8aa3b, v3\n.Lfunc_end0:\n")
    assert close_vgpr_result_reads(asm) == {"_Zbaz": 1}
    safe = asm.replace("\tv_mul", "\ts_nop 7\n\ts_nop 4\n\tv_mul")
    assert close_vgpr_result_reads(safe) == {}



def _sregs(text: str) -> set[int]:
    out = set()
    for m in re.finditer(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b", text):
        lo = int(m.group(1) or m.group(3))
        hi = int(m.group(2) or m.group(3))
        out.update(range(lo, hi + 1))
    return out


def valu_sgpr_to_vmem(asm: str, states: int = 5) -> dict[str, int]:
    """A VALU write of an SGPR (``v_readlane`` / ``v_readfirstlane`` / an
    ``_e64`` compare into an SGPR pair) read by a vector-memory instruction as
    descriptor, offset or base within ``states`` wait states.  hipcc pads this
    for its own loads, not for an inline-asm ``buffer_load ... lds``: with the
    causal forward's SGPRs spilled to VGPR lanes, a descriptor word restored by
    ``v_readlane`` right before the DMA was read stale (keys lost from O: the
    record count; a memory fault: the base)."""
    bad = {}
    for name in re.findall(r"^(_Z[^\s:]+):", asm, re.M):
        i = asm.find(name + ":")
        j = asm.find(".Lfunc_end", i)
        body = [ln.split(";")[0].strip() for ln in asm[i:j].split("\n")]
        body = [ln for ln in body if ln and not ln.startswith(".") and not ln.endswith(":")]
        pend: dict[int, int] = {}
        n = 0
        for ln in body:
            op, _, rest = ln.partition(" ")
            m = re.match(r"s_nop (\d+)", ln)
            step = int(m.group(1)) + 1 if m else 1
            if op.startswith(("buffer_", "global_", "flat_", "scratch_")) and \
                    any(r in pend for r in _sregs(rest)):
                n += 1
            pend = {r: c + step for r, c in pend.items() if c + step < states}
            if op.startswith(("v_readlane", "v_readfirstlane")) or \
                    (op.startswith("v_cmp") and op.endswith("_e64")):
                for r in _sregs(rest.split(",")[0]):
                    pend[r] = 0
            if op in ("s_branch", "s_endpgm", "s_setpc_b64"):
                pend = {}
        if n:
            bad[name] = n
    return bad


def test_detector_flags_a_stale_descriptor_word():
    asm = ("_Zdma:\n\tv_readlane_b32 s27, v225, 18\n\ts_nop 0\n"
           "\tbuffer_load_dwordx4 v137, s[24:27], s3 offen lds\n.Lfunc_end0:\n")
    assert valu_sgpr_to_vmem(asm) == {"_Zdma": 1}
    assert valu_sgpr_to_vmem(asm.replace("s_nop 0", "s_nop 4")) == {}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", ["attention.hip", "attention_bwd256.hip", "attention_fwd256.hip",
                                 "attention_dq256.hip", "gemm_bf16.hip", "gemm_bf16_layouts.hip"])
def test_asm_dma_reads_no_fresh_valu_sgpr(src, tmp_path):
    asm = _asm(src, str(tmp_path / (src + ".s")))
    assert "buffer_load" in asm
    assert valu_sgpr_to_vmem(asm) == {}


def asm_load_dests_touched(asm: str, kernel_re: str, wait: str) -> list[str]:
    """Instructions that read or write the destination registers of the
    inline-asm ``global_load`` run of a kernel's prologue before ``wait``
    (the asm ``s_waitcnt`` that covers them).  hipcc counts an asm load's
    destination as written at ``;;#ASMEND`` and may copy or reuse it before
    the data lands (seen: a branch merge copied all 16 Q registers)."""
    bad = []
    for name in re.findall(r"^(_Z[^\s:]+):", asm, re.M):
        if not re.search(kernel_re, name):
            continue
        i = asm.find(name + ":")
        j = asm.find(".Lfunc_end", i)
        body = [ln.split(";")[0].strip() for ln in asm[i:j].split("\n")]
        body = [ln for ln in body if ln and not ln.startswith(".") and not ln.endswith(":")]
        k0 = next(k for k, ln in enumerate(body) if ln.startswith("global_load"))
        dst: set[int] = set()
        for ln in body[k0:]:
            if ln.startswith(wait):
                break
            op, _, rest = ln.partition(" ")
            if op.startswith("global_load"):
                d, _, srcs = rest.partition(",")
                if _regs(srcs) & dst:
                    bad.append(ln)
                dst |= _regs(d)
            elif _regs(rest) & dst:
                bad.append(ln)
    return bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_dq256_prologue_loads_untouched_before_their_wait(tmp_path):
    """attention_dq256.hip issues its lse loads as inline asm beside the
    LDS-DMA of dO / O; nothing may read or copy their destinations before the
    wait."""
    asm = _asm("attention_dq256.hip", str(tmp_path / "d.s"), ("-fno-slp-vectorize",))
    assert asm_load_dests_touched(asm, "mxk_attn_bwd_dq256_kernel", "s_waitcnt vmcnt(0)") == []


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_fwd256_prologue_q_loads_untouched_before_their_wait(tmp_path):
    asm = _asm("attention_fwd256.hip", str(tmp_path / "f.s"))
    assert asm_load_dests_touched(asm, "mxk_attn_fwd256_kernel", "s_waitcnt vmcnt(16)") == []


_TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32", "v_cos_f32")


def trans_result_read_next(asm: str) -> list[str]:
    """An instruction reading the result of the transcendental right before
    it (gfx950 needs one wait state there; hipcc pads its own instructions
    but not an inline-asm reader).  Seen: the 256-row forward's asm row-sum
    adds behind the v_exp_f32 of their score - wrong sums in the lanes the
    transcendental unit had not finished."""
    bad = []
    body = [ln.split(";")[0].strip() for ln in asm.split("\n")]
    body = [ln for ln in body if ln and not ln.startswith(".") and not ln.endswith(":")]
    for k, ln in enumerate(body[:-1]):
        op, _, rest = ln.partition(" ")
        if not op.startswith(_TRANS):
            continue
        nxt = body[k + 1]
        if nxt.startswith("s_nop") or "," not in nxt:
            continue
        if _regs(nxt.split(",", 1)[1]) & _regs(rest.split(",")[0]):
            bad.append(ln + " | " + nxt)
    return bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", ["attention.hip", "attention_bwd256.hip", "attention_fwd256.hip",
                                 "attention_dq256.hip"])
def test_no_asm_read_of_a_fresh_transcendental(src, tmp_path):
    asm = _asm(src, str(tmp_path / "t.s"))
    assert trans_result_read_next(asm) == []


def test_detector_flags_a_fresh_transcendental_read():
    asm = "\tv_exp_f32_e32 v26, v26\n\tv_add_f32_e32 v4, v4, v26\n\tv_exp_f32_e32 v2, v2\n\ts_nop 0\n\tv_add_f32_e32 v4, v4, v2\n"
    assert trans_result_read_next(asm) == ["v_exp_f32_e32 v26, v26 | v_add_f32_e32 v4, v4, v26"]


def test_detector_flags_a_copy_of_an_inflight_load():
    asm = ("_Zq:\n\tglobal_load_dwordx4 v[2:5], v[30:31], off\n\tv_mov_b64_e32 v[70:71], v[2:3]\n"
           "\ts_waitcnt vmcnt(16)\n.Lfunc_end0:\n")
    assert asm_load_dests_touched(asm, "_Zq", "s_waitcnt vmcnt(16)") == ["v_mov_b64_e32 v[70:71], v[2:3]"]


def valu_write_then_mfma_read(asm: str, states: int = 2) -> dict[str, int]:
    """An inline-asm MFMA reading (as A, B or C) a VGPR that a VALU
    instruction wrote fewer than ``states`` wait states before (hipcc pads
    this only for its own MFMAs).  Seen: merging the 256-key backward's two
    S / dP phases put the VALU copies of the initial accumulators right in
    front of the tile-1 chains (dK off by 9.6)."""
    bad = {}
    for name in re.findall(r"^(_Z[^\s:]+):", asm, re.M):
        i = asm.find(name + ":")
        j = asm.find(".Lfunc_end", i)
        body = [ln.split(";")[0].strip() for ln in asm[i:j].split("\n")]
        body = [ln for ln in body if ln and not ln.startswith(".") and not ln.endswith(":")]
        pend: dict[int, int] = {}
        n = 0
        for ln in body:
            op, _, rest = ln.partition(" ")
            m = re.match(r"s_nop (\d+)", ln)
            step = int(m.group(1)) + 1 if m else 1
            if op.startswith("v_mfma"):
                srcs = rest.partition(",")[2]
                if any(pend.get(r, states) < states for r in _regs(srcs)):
                    n += 1
                pend = {r: c + step for r, c in pend.items() if c + step < states}
                continue
            pend = {r: c + step for r, c in pend.items() if c + step < states}
            if op.startswith("v_") and not op.startswith(("v_accvgpr_write", "v_readlane",
                                                          "v_readfirstlane", "v_cmp")):
                dst = rest.partition(",")[0]
                for r in _regs(dst):
                    pend[r] = 0
            if op in ("s_branch", "s_endpgm", "s_setpc_b64"):
                pend = {}
        if n:
            bad[name] = n
    return bad


def _aregs(text: str) -> set[int]:
    out = set()
    for m in re.finditer(r"\ba\[(\d+):(\d+)\]|\ba(\d+)\b", text):
        lo = int(m.group(1) or m.group(3))
        hi = int(m.group(2) or m.group(3))
        out.update(range(lo, hi + 1))
    return out


def agpr_write_then_mfma_read(asm: str, states: int = 2) -> dict[str, int]:
    """An inline-asm MFMA reading (as A, B or C) an AGPR that a
    v_accvgpr_write / v_accvgpr_mov wrote fewer than ``states`` wait states
    before.  Seen: the register allocator shuffling the dQ^T tiles between the
    loop and the tail's own MFMA instance (attention_dq256.hip) wrote a48 -
    register 0 of a tile - right in front of the MFMA accumulating into
    a[48:63]: that register alone missed its earlier sum in every block."""
    bad = {}
    for name in re.findall(r"^(_Z[^\s:]+):", asm, re.M):
        i = asm.find(name + ":")
        j = asm.find(".Lfunc_end", i)
        body = [ln.split(";")[0].strip() for ln in asm[i:j].split("\n")]
        body = [ln for ln in body if ln and not ln.startswith(".") and not ln.endswith(":")]
        pend: dict[int, int] = {}
        n = 0
        for ln in body:
            op, _, rest = ln.partition(" ")
            m = re.match(r"s_nop (\d+)", ln)
            step = int(m.group(1)) + 1 if m else 1
            if op.startswith("v_mfma"):
                srcs = rest.partition(",")[2]
                if any(pend.get(r, states) < states for r in _aregs(srcs)):
                    n += 1
                pend = {r: c + step for r, c in pend.items() if c + step < states}
                continue
            pend = {r: c + step for r, c in pend.items() if c + step < states}
            if op.startswith(("v_accvgpr_write", "v_accvgpr_mov")):
                for r in _aregs(rest.partition(",")[0]):
                    pend[r] = 0
            if op in ("s_branch", "s_endpgm", "s_setpc_b64"):
                pend = {}
        if n:
            bad[name] = n
    return bad


def test_detector_flags_a_fresh_accumulator_copy():
    asm = ("_Zd:\n\tv_accvgpr_write_b32 a48, v32\n"
           "\tv_mfma_f32_32x32x16_bf16 a[48:63], v[4:7], v[0:3], a[48:63]\n.Lfunc_end0:\n")
    assert agpr_write_then_mfma_read(asm) == {"_Zd": 1}
    assert agpr_write_then_mfma_read(asm.replace("\tv_mfma", "\ts_nop 1\n\tv_mfma")) == {}


def test_detector_flags_a_fresh_mfma_operand():
    asm = ("_Zc:\n\tv_mov_b64_e32 v[32:33], v[16:17]\n"
           "\tv_mfma_f32_32x32x16_bf16 v[32:47], v[0:3], v[4:7], v[32:47]\n.Lfunc_end0:\n")
    assert valu_write_then_mfma_read(asm) == {"_Zc": 1}
    assert valu_write_then_mfma_read(asm.replace("\tv_mfma", "\ts_nop 1\n\tv_mfma")) == {}


def scratch_in_loops(asm: str) -> dict[str, int]:
    """Scratch (spill) instructions between a loop header label and the last
    branch back to it, per kernel (linear layout: LLVM keeps a loop's blocks
    contiguous)."""
    bad = {}
    for name in re.findall(r"^(_Z[^\s:]+):", asm, re.M):
        i = asm.find(name + ":")
        j = asm.find(".Lfunc_end", i)
        lines = asm[i:j].split("\n")
        n = 0
        for k, ln in enumerate(lines):
            m = re.match(r"^(\.LBB\d+_\d+):.*Loop Header", ln)
            if not m:
                continue
            lab = m.group(1)
            ends = [e for e in range(k + 1, len(lines))
                    if re.match(r"\s*s_c?branch\S*\s+" + re.escape(lab) + r"\b", lines[e])]
            if ends:
                n += sum(1 for e in range(k, ends[-1]) if "scratch_" in lines[e].split(";")[0])
        if n:
            bad[name] = n
    return bad


def test_detector_flags_a_reload_in_a_loop():
    asm = ("_Zl:\n.LBB0_1:  ; =>This Inner Loop Header: Depth=1\n"
           "\tscratch_load_dword v1, off, off\n\ts_cbranch_scc1 .LBB0_1\n"
           "\tscratch_load_dword v2, off, off\n.Lfunc_end0:\n")
    assert scratch_in_loops(asm) == {"_Zl": 1}

@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", ["attention_bwd256.hip", "attention_fwd256.hip",
                                 "attention_dq256.hip"])
def test_attention_bwd256_asm_mfma_hazards_and_spills(src, tmp_path):
    """attention_bwd256.hip / attention_fwd256.hip / attention_dq256.hip: the
    accumulated tiles (dK^T / dV^T; O^T; dQ^T) pinned to AGPRs and S / dP (S^T) to VGPRs by
    inline-asm MFMAs; no early read of either, and no spill (their LDS-DMA
    ring waits are counted vmcnt waits)."""
    asm = _asm(src, str(tmp_path / (src + ".s")))
    assert "v_mfma" in asm
    assert close_accumulator_reads(asm) == {}
    assert close_vgpr_result_reads(asm) == {}
    assert valu_write_then_mfma_read(asm) == {}
    assert agpr_write_then_mfma_read(asm) == {}
    # no scratch access inside a loop (a reload there is a vector-memory op
    # the counted vmcnt waits of the LDS-DMA rings do not expect); a spill
    # stored before the loop and reloaded after it is harmless
    assert scratch_in_loops(asm) == {}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,flags", [("gemm_bf16.hip", ()), ("gemm_bf16_layouts.hip", ()),
                                       ("experiments/gemm_tn_exp.hip", ("-DMXK_GEMM_EXPERIMENTS",))])
def test_no_accumulator_read_right_after_asm_mfma(src, flags, tmp_path):
    asm = _asm(src, str(tmp_path / (src.replace("/", "_") + ".s")), flags)
    assert "v_mfma" in asm
    assert close_accumulator_reads(asm) == {}


def test_detector_flags_a_close_read():
    asm = ("_Zfoo:\n\tv_mfma_f32_16x16x32_bf16 a[0:3], v[0:3], v[4:7], a[0:3]\n"
           "\ts_add_u32 s0, s0, 1\n\tv_accvgpr_read_b32 v8, a2\n.Lfunc_end0:\n")
    assert close_accumulator_reads(asm) == {"_Zfoo": 1}
    safe = asm.replace("\ts_add_u32 s0, s0, 1\n", "\ts_nop 7\n\ts_nop 7\n")
    assert close_accumulator_reads(safe) == {}


def test_detector_flags_a_close_accumulator_spill():
    asm = ("_Zbar:\n\tv_mfma_f32_16x16x32_bf16 a[252:255], v[0:3], v[4:7], a[252:255]\n"
           "\ts_mov_b32 s0, 1\n\tscratch_store_dwordx4 off, a[252:255], off offset:4\n"
           ".Lfunc_end0:\n")
    assert close_accumulator_reads(asm) == {"_Zbar": 1}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,flags", [("gemm_bf16.hip", ()), ("gemm_bf16_layouts.hip", ()),
                                       # the trickle-store kernels are experiments-only
                                       ("experiments/gemm_tn_exp.hip", ("-DMXK_GEMM_EXPERIMENTS",)),
                                       ("gemm_bf16_layouts.hip", ("-DMXK_GEMM_EXPERIMENTS",))])
def test_counted_wait_gemms_do_not_spill(src, flags, tmp_path):
    """The GEMM loops wait for their LDS-DMA stages with COUNTED vmcnt waits
    (all but the N youngest vector-memory ops).  A register spill or reload
    is a vector-memory op the count does not expect: a reload inside the loop
    lets the wait pass one DMA piece early (seen: the trickle-store layout
    kernel's wgrad instance at 10 spills gave wrong tiles, the 9 without
    spills were exact).  Every shipped counted-wait GEMM kernel: no spills."""
    asm = _asm(src, str(tmp_path / (src.replace("/", "_") + ".s")), flags)
    names = re.findall(r"^\s+\.name:\s+(_Z\S+)", asm, re.M)
    counts = [int(x) for x in re.findall(r"\.vgpr_spill_count:\s+(\d+)", asm)]
    assert len(names) == len(counts) and names
    # production: every counted-wait GEMM; experiments build: the trickle-store
    # kernels (the round-2 persistent w4ip records are known to spill)
    pat = re.compile(r"mxk_gemm_bf16_(tn_w4t|x2t_kernel)" if flags else
                     r"mxk_gemm_bf16_(tn_w4t|x2t_kernel|tn_w4j|x2_kernel)")
    checked = {n: c for n, c in zip(names, counts) if pat.search(n)}
    assert checked, "no counted-wait GEMM kernel found"
    assert {n: c for n, c in checked.items() if c} == {}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("kernel", ["w13_swiglu"])
def test_epilogue_spills_stay_out_of_the_dma_loop(kernel, tmp_path):
    """The fused up-projection keeps 3 spill slots for its epilogue; none of
    them may sit inside the counted-wait K loop (a scratch op there would be a
    vector-memory op the loop's vmcnt counts do not expect).  The tail
    K-tiles after the loop wait with vmcnt(0), which also covers a spill."""
    asm = _asm("gemm_bf16.hip", str(tmp_path / "g.s"))
    names = re.findall(r"^(_Z\S*mxk_gemm_bf16_%s\S*):" % kernel, asm, re.M)
    assert names
    for name in names:
        body = asm[asm.index(name + ":"):]
        body = body[:body.index("s_endpgm")]
        lines = body.split("\n")
        heads = [i for i, l in enumerate(lines) if "Inner Loop Header" in l]
        assert heads, "no K loop found"
        for h in heads:
            label = lines[h].split(":")[0]
            end = next(i for i in range(h + 1, len(lines))
                       if "s_cbranch" in lines[i] and lines[i].rstrip().endswith(label))
            assert not [l for l in lines[h:end + 1] if "scratch_" in l], (name, label)
