#!/usr/bin/env python3
"""1-GPU rehearsal of compute / collective co-residency.

At n > 1 the ZeRO-1 reduce-scatter runs under the backward, and RCCL's
kernels keep a set of CUs busy for as long as it lasts.  Here a copy kernel
holding k CUs (native/kernels/contention.hip; --placement spread: k
workgroups dealt over the XCDs like RCCL's channels, masked: a CU-masked
stream on CUs [0, k)) runs through every backward of the Llama-3-8B step
(seq 2048, micro-batch 8, bf16, AdamW - the BASELINE config 5 step at world
1), and the step is timed

  base      no streamer
  blind     streamer on k CUs, GEMM planner unaware (plans for 256 CUs)
  aware     streamer on k CUs, mxk_gemm_set_reserved_cus(k): rounds and the
            split tail are sized for the 256 - k CUs left
  excl_*    the same with the GEMMs in exclusive mode (mxk_gemm_set_exclusive:
            each GEMM workgroup claims its CU's whole LDS, so the streamer's
            workgroups cannot share a CU with a GEMM tile and slow it; they
            take whole CUs between tiles instead)

for k in --cus.  The streamer is paced to --gbps (copy traffic, read +
write; default 700 GB/s, what an 8-rank ring reduce-scatter of the bf16
gradient buckets puts on one GPU's HBM over xGMI) so that it takes CUs the
way a collective does without also taking most of HBM; --gbps 0 lets it run
flat out (a bandwidth hog, not a collective).  Prints one RESULT json per
(k, placement, mode): ms/step, the backward's ms (the streamer runs beside
it) and both slowdowns against base.  The criterion is the
backward slowdown <= k/256 + 2 %.

    python scripts/contention_bench.py --cus 16,32,64 [--gbps 700] [--steps 6] [--layers N]
"""
import argparse
import itertools
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxk8s.models.llama import LlamaConfig  # noqa: E402
from mxk8s.ops import _lib, gemm  # noqa: E402
from mxk8s.utils import roctx  # noqa: E402
from mxk8s.train.ddp_llama import build, use_tuned_gemms  # noqa: E402


def cu_mask_map(dev) -> dict:
    """mask bit -> (XCC, SE, SH, CU) of the CU it names: a one-bit CU-masked
    stream per bit runs mxk_cu_probe (contention.hip) and reads back HW_ID /
    XCC_ID of where its workgroups landed."""
    import ctypes
    L = _lib.lib()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nw = 16
    out = torch.zeros(2 * nw, dtype=torch.int32, device=dev)
    res = {}
    for b in range(cus):
        h = ctypes.c_void_p()
        bits = (ctypes.c_int * 1)(b)
        _lib.check(L.mxk_stream_create_cu_masked_bits(bits, 1, ctypes.byref(h)), "masked stream")
        _lib.check(L.mxk_cu_probe(out.data_ptr(), nw, 20000, h.value), "cu probe")
        torch.cuda.synchronize()
        L.mxk_stream_destroy(h.value)
        v = out.cpu().tolist()
        places = {(v[2 * i + 1] & 0xF, (v[2 * i] >> 13) & 7, (v[2 * i] >> 12) & 1, (v[2 * i] >> 8) & 15)
                  for i in range(nw)}
        res[b] = sorted(places)
    return res


def xcd_balanced_bits(k: int, cmap: dict) -> list:
    """k mask bits, k/8 on each XCC, from the probed map (one CU per bit)."""
    per = {}
    for b in sorted(cmap):
        if len({p[0] for p in cmap[b]}) == 1:
            per.setdefault(cmap[b][0][0], []).append(b)
    if len(per) != 8 or any(len(v) < k // 8 for v in per.values()):
        raise SystemExit("CU mask bits do not name single XCDs on this device (see CUMAP); "
                         "no xcd placement")
    return sorted(b for x in sorted(per) for b in per[x][:k // 8])


class Streamer:
    """HBM copy kernel holding k CUs.

    placement "spread" (default, what RCCL's kernels look like): k
    workgroups of 256 threads on an ordinary high-priority stream; workgroups
    are dealt round-robin over the 8 XCDs, so k/8 CUs of every XCD are held.
    placement "masked": 4k workgroups on a stream CU-masked to CUs [0, k) -
    all of them on the first XCD(s), the worst case for a GEMM whose tiles
    are dealt evenly over the XCDs (that XCD then finishes last).
    placement "xcd": 4k workgroups on a stream CU-masked to k/8 CUs of every
    XCD, the bits chosen from the probed mask -> CU map (cu_mask_map) - how a
    collective confined to a CU partition would sit."""

    def __init__(self, k: int, dev, mib: int = 512, placement: str = "spread", cmap=None):
        import ctypes
        self.k = k
        self.L = _lib.lib()
        self.owned = placement in ("masked", "xcd")
        if self.owned:
            h = ctypes.c_void_p()
            if placement == "xcd":
                assert k % 8 == 0, "xcd placement needs k % 8 == 0"
                bits = xcd_balanced_bits(k, cmap if cmap is not None else cu_mask_map(dev))
                arr = (ctypes.c_int * len(bits))(*bits)
                _lib.check(self.L.mxk_stream_create_cu_masked_bits(arr, len(bits), ctypes.byref(h)),
                           "cu-masked stream")
            else:
                _lib.check(self.L.mxk_stream_create_cu_masked(0, k, 0, ctypes.byref(h)), "cu-masked stream")
            self.handle = h.value
            self.stream = torch.cuda.ExternalStream(self.handle, device=dev)
            self.nwg = 4 * k
        else:
            self.stream = torch.cuda.Stream(device=dev, priority=-1)
            self.handle = self.stream.cuda_stream
            self.nwg = k
        n = mib * 2 ** 20
        self.src = torch.empty(n, dtype=torch.uint8, device=dev).fill_(1)
        self.dst = torch.empty(n, dtype=torch.uint8, device=dev)
        self.iters = 1
        self.pace = 0

    def launch(self):
        _lib.check(self.L.mxk_hbm_stream_paced(self.src.data_ptr(), self.dst.data_ptr(),
                                               self.src.numel(), self.iters, self.nwg, self.pace,
                                               self.handle), "hbm stream")

    def time_one(self) -> float:
        """ms of one pass over the buffer, alone on the GPU."""
        self.iters = 1
        with torch.cuda.stream(self.stream):
            self.launch()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                self.launch()
            e.record()
            e.synchronize()
        return s.elapsed_time(e) / 3

    def gbps(self, ms: float) -> float:
        return 2 * self.src.numel() / ms / 1e6

    def calibrate(self, target_ms: float, gbps: float = 0.0, gb_per_step: float = 0.0):
        """Pace to <= gbps (0: unpaced), then enough passes to cover target_ms,
        or (gb_per_step > 0) to move that many GB of copy traffic per step."""
        self.pace = 0
        one = self.time_one()
        if gbps > 0 and self.gbps(one) > gbps:
            lo, hi = 0, 1
            while True:
                self.pace = hi
                one = self.time_one()
                if self.gbps(one) <= gbps or hi >= 4096:
                    break
                lo, hi = hi, hi * 2
            while hi - lo > 1:                 # smallest pace within the target
                self.pace = (lo + hi) // 2
                t = self.time_one()
                if self.gbps(t) <= gbps:
                    hi, one = self.pace, t
                else:
                    lo = self.pace
            self.pace = hi
        if gb_per_step > 0:
            self.iters = max(1, int(round(gb_per_step * 1e9 / (2 * self.src.numel()))))
        else:
            self.iters = max(1, int(round(target_ms / one)))
        return one

    def close(self):
        torch.cuda.synchronize()
        if self.owned:
            self.L.mxk_stream_destroy(self.handle)


def step(model, ddp, opt, tokens, streamer=None, times=None):
    cur = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    loss = model.loss(tokens)
    ev[1].record()
    if streamer is not None:
        streamer.stream.wait_event(ev[1])         # starts with the backward
        with torch.cuda.stream(streamer.stream):
            streamer.launch()
    loss.backward()
    ddp.finish_grad_sync()
    ev[2].record()
    opt.step()
    ddp.zero_grad()
    if streamer is not None:
        cur.wait_stream(streamer.stream)          # like a collective the step waits for
    if times is not None:
        times.append(ev)
    return loss


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--cus", default="16,32,64")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--layers", type=int, default=None, help="fewer layers (quick check only)")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--micro-batch", type=int, default=8)
    ap.add_argument("--placement", default="spread", help="comma list: spread, xcd, masked")
    ap.add_argument("--map-only", action="store_true", help="print the CU-mask bit map and exit")
    ap.add_argument("--gb-per-step", type=float, default=0.0,
                    help="streamer traffic per step in GB (read + write); 0: it runs through the "
                         "whole backward.  28 is an 8-rank ZeRO-1 gradient reduce-scatter of "
                         "Llama-3-8B (16 GB of bf16 gradients, 7/8 of it read and written once)")
    ap.add_argument("--modes", default="blind,aware,excl_blind,excl_aware",
                    help="comma list: blind, aware, excl_blind, excl_aware")
    ap.add_argument("--base-steps", type=int, default=None,
                    help="steps of the base run (default --steps; its backward time calibrates "
                         "the streamer)")
    ap.add_argument("--gbps", default="700",
                    help="comma list of streamer copy rates (read + write, GB/s); 0: unpaced. "
                         "A few GB/s isolates the CUs the streamer holds from the HBM it takes")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cmap = None
    if a.map_only or "xcd" in a.placement:
        cmap = cu_mask_map(dev)
        xccs = {}
        for b, pl in cmap.items():
            for p in pl:
                xccs.setdefault(p[0], set()).add(b)
        print("CUMAP " + json.dumps({"bits_per_xcc": {x: len(v) for x, v in sorted(xccs.items())},
                                     "map": {b: cmap[b] for b in range(len(cmap))}}), flush=True)
        if a.map_only:
            return 0
    use_tuned_gemms()
    cfg = LlamaConfig.llama3_8b()
    if a.layers:
        cfg.n_layers = a.layers
    model, ddp, opt = build(cfg, dev, 512.0, zero=False)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    batches = [torch.randint(0, cfg.vocab_size, (a.micro_batch, a.seq_len + 1), device=dev, generator=g)
               for _ in range(2)]

    def timed(streamer=None, label="base"):
        for i in range(a.warmup):
            step(model, ddp, opt, batches[i % 2], streamer)
        torch.cuda.synchronize()
        walls, evs = [], []
        with roctx.range(f"contention.{label}"):     # kernel traces split by these ranges
            for i in range(a.steps):
                t0 = time.perf_counter()
                step(model, ddp, opt, batches[i % 2], streamer, evs)
                torch.cuda.synchronize()
                walls.append((time.perf_counter() - t0) * 1e3)
        bwd = statistics.median(e[1].elapsed_time(e[2]) for e in evs)
        return statistics.median(walls), bwd

    gemm.set_reserved_cus(0)
    base, base_bwd = timed()
    print("RESULT " + json.dumps({"k": 0, "mode": "base", "ms_per_step": round(base, 2),
                                  "backward_ms": round(base_bwd, 2), "layers": cfg.n_layers}),
          flush=True)
    for placement, gbps, k in itertools.product(a.placement.split(","),
                                                [float(x) for x in a.gbps.split(",") if x],
                                                [int(x) for x in a.cus.split(",") if x]):
        st = Streamer(k, dev, placement=placement, cmap=cmap)
        one = st.calibrate(base_bwd, gbps, a.gb_per_step)
        for mode in a.modes.split(","):
            gemm.set_reserved_cus(k if mode.endswith("aware") else 0)
            gemm.set_exclusive(mode.startswith("excl"))
            ms, bwd = timed(st, f"k{k}.{placement}.{gbps:g}.{mode}")
            ideal = k / 256 * base_bwd / base
            bslow = bwd / base_bwd - 1
            print("RESULT " + json.dumps({
                "k": k, "placement": placement, "gbps_target": gbps, "mode": mode,
                "gb_per_step": a.gb_per_step or None,
                "ms_per_step": round(ms, 2),
                "backward_ms": round(bwd, 2), "slowdown": round(ms / base - 1, 4),
                "backward_slowdown": round(bslow, 4), "ideal_slowdown": round(ideal, 4),
                "criterion": round(k / 256 + 0.02, 4), "meets": bslow <= k / 256 + 0.02,
                "streamer_gbps_alone": round(st.gbps(one), 1), "streamer_pace": st.pace,
                "streamer_iters": st.iters, "streamer_ms_per_iter_alone": round(one, 3),
                "available_cus": gemm.available_cus()}), flush=True)
        gemm.set_reserved_cus(0)
        gemm.set_exclusive(False)
        st.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
