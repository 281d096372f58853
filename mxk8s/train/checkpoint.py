"""Checkpoint / resume of the flat-buffer trainer (SURVEY.md §5
"Checkpoint / resume": the reference has none; its only resumable sequence is
the manual reboot gate, /root/reference/README.md:70-84).

Everything the trainer owns lives in a handful of flat buffers
(:class:`~mxk8s.parallel.ddp.FlatParamSpace`, the AdamW master / moment
buffers), so a checkpoint is a few large contiguous tensors — no per-parameter
state dicts, no pickles.  Format ``mxk8s-flat-v2``:

  <dir>/step-<N>/params.safetensors        bf16 parameters (rank 0; identical on all ranks)
  <dir>/step-<N>/optim-rank<r>.safetensors fp32 master / exp_avg / exp_avg_sq of rank r
                                           (its ZeRO-1 shard, or the full buffers when
                                           the optimizer is replicated — then rank 0 only)
  <dir>/meta.json                          commit record: step, world size, layout
                                           fingerprint, sharding, which step-<N>, and
                                           the committed step-<N> history

Every save writes a NEW step directory; ``meta.json`` — written by rank 0
after a barrier that every rank reaches once its shard is on disk, then
renamed into place — is what makes it current.  An interrupted save leaves
the previous step directory and the previous ``meta.json`` untouched, so the
job resumes from the last complete checkpoint.  ``meta.json`` also lists the
committed step directories (``history``); after each commit the ``keep``
newest of those are retained and every other step directory is removed —
older commits and the uncommitted leftovers of interrupted saves alike, so a
stale higher-numbered directory never evicts a usable checkpoint.
Every shard also carries its own ``step_count`` / ``layout`` / ``save_step``,
which ``load`` checks against ``meta.json``.

Loading checks the layout fingerprint (parameter shapes, offsets, bucket
padding) and, for sharded state, the world size, and refuses mismatches.
Format ``mxk8s-flat-v1`` directories (shards directly in ``<dir>``) still
load; their shards may predate the ``save_step`` tag, which is then not
checked.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Optional

import torch
from safetensors.torch import load_file, save_file

from ..parallel import dist as mxdist


def layout_fingerprint(space) -> str:
    h = hashlib.sha256()
    for p, o in zip(space.params, space.offsets):
        h.update(f"{tuple(p.shape)}@{o};".encode())
    h.update(f"numel={space.numel};dtype={space.dtype}".encode())
    return h.hexdigest()[:16]


def _atomic_save(tensors: dict, path: str, meta: Optional[dict] = None) -> None:
    tmp = path + ".tmp"
    save_file({k: v.detach().contiguous().cpu() for k, v in tensors.items()}, tmp,
              metadata={k: str(v) for k, v in (meta or {}).items()})
    os.replace(tmp, path)


def _check_shard(path: str, meta: dict, want: dict, legacy: bool = False) -> None:
    """A shard's own safetensors metadata must match the commit record (v1
    shards written before the save_step tag existed skip that key)."""
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        have = f.metadata() or {}
    bad = {k: (have.get(k), v) for k, v in want.items()
           if have.get(k) != v and not (legacy and k == "save_step" and k not in have)}
    if bad:
        raise ValueError(f"{path}: shard does not match meta.json (step {meta['step']}): "
                         + ", ".join(f"{k}={h!r} expected {w!r}" for k, (h, w) in bad.items())
                         + " — the shard was overwritten after meta.json was committed")


FORMAT = "mxk8s-flat-v2"
LEGACY_FORMAT = "mxk8s-flat-v1"


def step_dirname(step: int) -> str:
    return f"step-{step:09d}"


def _write_meta(ckpt_dir: str, meta: dict) -> None:
    tmp = os.path.join(ckpt_dir, "meta.json.tmp")
    with open(tmp, "w") as f:
        json.dump(meta, f, indent=1)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, os.path.join(ckpt_dir, "meta.json"))


def _read_meta(ckpt_dir: str) -> Optional[dict]:
    try:
        with open(os.path.join(ckpt_dir, "meta.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _complete_dirs(ckpt_dir: str, shards: Optional[int] = None) -> list[str]:
    """Step directories that hold a complete shard set, oldest first
    (zero-padded step names): params plus every optimizer shard
    ``optim-rank0 .. optim-rank<shards-1>`` (``shards``: the current save's
    shard count, 1 when the optimizer is replicated).  An interrupted
    sharded save - rank 0's files on disk, a later rank's missing - is not
    complete and never takes a retention slot.  ``shards=None`` (no current
    save to compare with) only asks for params plus ``optim-rank0``."""
    out = []
    want = [f"optim-rank{r}.safetensors" for r in range(shards or 1)]
    for d in sorted(os.listdir(ckpt_dir)):
        full = os.path.join(ckpt_dir, d)
        if not (d.startswith("step-") and os.path.isdir(full)):
            continue
        names = set(os.listdir(full))
        if "params.safetensors" in names and all(w in names for w in want):
            out.append(d)
    return out


def _history(prev: Optional[dict], current: str, keep: int,
             ckpt_dir: Optional[str] = None, shards: Optional[int] = None) -> list[str]:
    """Committed step directories, oldest first, ending with ``current``:
    the previous commit record's history (or its single ``path`` for records
    written before the history existed), truncated to the ``keep`` newest.
    When no usable record exists (missing, unreadable, another format, or a
    record without ``history``) and ``ckpt_dir`` is given, fall back to the
    newest ``keep`` directories with a complete shard set, so a lost
    meta.json never makes the prune delete every earlier commit."""
    hist = []
    if prev and prev.get("format") == FORMAT and prev.get("history"):
        hist = list(prev["history"])
    else:
        if prev and prev.get("format") == FORMAT and prev.get("path"):
            hist = [prev["path"]]
        if ckpt_dir is not None:
            hist = sorted(set(hist) | set(_complete_dirs(ckpt_dir, shards)))
    hist = [h for h in hist if h != current] + [current]
    return hist[-max(1, keep):]


def _prune(ckpt_dir: str, history: list[str]) -> None:
    """Remove every step directory that is not one of the retained COMMITTED
    ones: older commits beyond ``keep`` and uncommitted directories left by
    an interrupted save (never counted toward ``keep``, whatever their step
    number).  Deleting more than one complete-looking directory at once is
    logged: that only happens after ``keep`` was lowered or a record was
    lost."""
    import shutil
    import sys
    victims = [d for d in os.listdir(ckpt_dir)
               if d.startswith("step-") and d not in history
               and os.path.isdir(os.path.join(ckpt_dir, d))]
    complete = set(_complete_dirs(ckpt_dir)) & set(victims)
    if len(complete) > 1:
        print(f"mxk8s.checkpoint: pruning {len(complete)} complete step directories "
              f"{sorted(complete)} (retained: {history})", file=sys.stderr)
    for d in victims:
        shutil.rmtree(os.path.join(ckpt_dir, d), ignore_errors=True)


def save(ckpt_dir: str, ddp, opt, step: int, keep: int = 2) -> None:
    """Collective: every rank calls it (rank 0 writes params + the commit record)."""
    world, rank, _ = mxdist.world_info()
    sharded = bool(getattr(ddp, "sharded", False))
    sub = step_dirname(step)
    sdir = os.path.join(ckpt_dir, sub)
    os.makedirs(sdir, exist_ok=True)
    fp = layout_fingerprint(ddp.space)
    if hasattr(opt, "synchronize"):
        opt.synchronize()      # pending side-stream updates (FlatAdamW overlap)
    if sharded or rank == 0:
        _atomic_save({"master": opt.master, "exp_avg": opt.exp_avg, "exp_avg_sq": opt.exp_avg_sq},
                      os.path.join(sdir, f"optim-rank{rank if sharded else 0}.safetensors"),
                      {"step_count": opt.step_count, "layout": fp, "save_step": step})
    if rank == 0:
        _atomic_save({"params": ddp.space.param_buf}, os.path.join(sdir, "params.safetensors"),
                     {"layout": fp, "save_step": step})
    # every shard is on disk before the commit record names this step
    mxdist.barrier()
    if rank == 0:
        history = _history(_read_meta(ckpt_dir), sub, keep, ckpt_dir,
                           shards=world if sharded else 1)
        _write_meta(ckpt_dir, {"step": step, "optimizer_step": opt.step_count, "world_size": world,
                               "sharded": sharded, "layout": fp, "numel": ddp.space.numel,
                               "format": FORMAT, "path": sub, "history": history})
        _prune(ckpt_dir, history)
    mxdist.barrier()


def load(ckpt_dir: str, ddp, opt) -> int:
    """Restore parameters and optimizer state; returns the saved step."""
    world, rank, _ = mxdist.world_info()
    if hasattr(opt, "synchronize"):
        opt.synchronize()      # no side-stream update may land after the restore
    with open(os.path.join(ckpt_dir, "meta.json")) as f:
        meta = json.load(f)
    fmt = meta.get("format")
    if fmt == FORMAT:
        sdir = os.path.join(ckpt_dir, meta["path"])
    elif fmt == LEGACY_FORMAT:
        sdir = ckpt_dir
    else:
        raise ValueError(f"{ckpt_dir}: not an mxk8s flat checkpoint (format {fmt!r})")
    fp = layout_fingerprint(ddp.space)
    if meta["layout"] != fp:
        raise ValueError(f"{ckpt_dir}: parameter layout {meta['layout']} != model layout {fp}")
    sharded = bool(getattr(ddp, "sharded", False))
    if meta["sharded"] != sharded or (sharded and meta["world_size"] != world):
        raise ValueError(f"{ckpt_dir}: saved with world_size={meta['world_size']} "
                         f"sharded={meta['sharded']}, running world_size={world} sharded={sharded}")
    dev = ddp.space.param_buf.device
    ppath = os.path.join(sdir, "params.safetensors")
    opath = os.path.join(sdir, f"optim-rank{rank if sharded else 0}.safetensors")
    legacy = fmt == LEGACY_FORMAT
    _check_shard(ppath, meta, {"layout": meta["layout"], "save_step": str(meta["step"])}, legacy)
    _check_shard(opath, meta, {"layout": meta["layout"], "save_step": str(meta["step"]),
                               "step_count": str(meta["optimizer_step"])}, legacy)
    params = load_file(ppath)["params"]
    with torch.no_grad():
        ddp.space.param_buf.copy_(params.to(dev))
        st = load_file(opath)
        opt.master.copy_(st["master"].to(dev))
        opt.exp_avg.copy_(st["exp_avg"].to(dev))
        opt.exp_avg_sq.copy_(st["exp_avg_sq"].to(dev))
    opt.step_count = int(meta["optimizer_step"])
    mxdist.barrier()
    return int(meta["step"])
