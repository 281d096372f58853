"""Checkpoint retention when the commit record is missing or old (ADVICE r4:
a lost meta.json must not make the prune delete every earlier commit)."""
import json
import os

from mxk8s.train import checkpoint as ck


def _mkstep(root, step, complete=True):
    d = os.path.join(root, ck.step_dirname(step))
    os.makedirs(d, exist_ok=True)
    open(os.path.join(d, "params.safetensors"), "w").close()
    if complete:
        open(os.path.join(d, "optim-rank0.safetensors"), "w").close()
    return os.path.basename(d)


def test_history_from_record(tmp_path):
    prev = {"format": ck.FORMAT, "path": "step-000000002",
            "history": ["step-000000001", "step-000000002"]}
    assert ck._history(prev, "step-000000003", 2, str(tmp_path)) == ["step-000000002",
                                                                    "step-000000003"]


def test_missing_meta_keeps_newest_complete(tmp_path, capsys):
    root = str(tmp_path)
    for s in (1, 2, 3):
        _mkstep(root, s)
    _mkstep(root, 4, complete=False)          # interrupted save: never retained
    cur = _mkstep(root, 5)
    hist = ck._history(ck._read_meta(root), cur, 3, root)
    assert hist == ["step-000000002", "step-000000003", cur]
    ck._prune(root, hist)
    left = sorted(d for d in os.listdir(root) if d.startswith("step-"))
    assert left == hist
    assert "pruning" not in capsys.readouterr().err   # one complete dir removed: no warning


def test_record_without_history_upgrades_without_dropping(tmp_path):
    root = str(tmp_path)
    for s in (1, 2):
        _mkstep(root, s)
    with open(os.path.join(root, "meta.json"), "w") as f:
        json.dump({"format": ck.FORMAT, "path": "step-000000002"}, f)
    cur = _mkstep(root, 3)
    hist = ck._history(ck._read_meta(root), cur, 3, root)
    assert hist == ["step-000000001", "step-000000002", cur]


def test_pruning_many_complete_dirs_is_logged(tmp_path, capsys):
    root = str(tmp_path)
    for s in (1, 2, 3, 4):
        _mkstep(root, s)
    ck._prune(root, ["step-000000004"])
    assert "pruning 3 complete step directories" in capsys.readouterr().err


def test_interrupted_sharded_save_is_not_complete(tmp_path):
    """a sharded save interrupted after rank 0's shards were written
    (rank 1's missing) must not take a retention slot and push a real commit
    into the prune."""
    root = str(tmp_path)
    for s in (1, 2):
        d = _mkstep(root, s)
        open(os.path.join(root, d, "optim-rank1.safetensors"), "w").close()
    _mkstep(root, 3)                          # rank 0 wrote, rank 1 did not
    cur = _mkstep(root, 4)
    open(os.path.join(root, cur, "optim-rank1.safetensors"), "w").close()
    assert ck._complete_dirs(root, shards=2) == ["step-000000001", "step-000000002", cur]
    hist = ck._history(None, cur, 3, root, shards=2)
    assert hist == ["step-000000001", "step-000000002", cur]
    ck._prune(root, hist)
    assert sorted(d for d in os.listdir(root) if d.startswith("step-")) == hist
