"""mxk8s.ops.embedding.Embedding: the dense weight gradient straight into
the flat gradient buffer (overwrite while fresh, add afterwards, then the
DDP readiness call), equal to nn.Embedding's."""
import torch

from mxk8s.ops.embedding import Embedding


def _pair(dtype=torch.float32):
    torch.manual_seed(0)
    e = Embedding(50, 8).to(dtype)
    ref = torch.nn.Embedding(50, 8).to(dtype)
    ref.weight.data.copy_(e.weight.data)
    t = torch.randint(0, 50, (3, 7))
    g = torch.randn(3, 7, 8).to(dtype)
    return e, ref, t, g


def test_plain_gradient_matches_nn_embedding():
    e, ref, t, g = _pair()
    assert torch.equal(e(t), ref(t))
    e(t).backward(g)
    ref(t).backward(g)
    assert torch.equal(e.weight.grad, ref.weight.grad)


def test_direct_gradient_overwrites_then_accumulates_and_notifies():
    for dtype in (torch.float32, torch.bfloat16):
        e, ref, t, g = _pair(dtype)
        ref(t).backward(g)
        calls = []
        w = e.weight
        w.main_grad = torch.full_like(w, 5.0)      # stale values: overwritten when fresh
        w._mxk_grad_fresh = True
        w._mxk_grad_ready = lambda: calls.append(1)
        e(t).backward(g)
        assert w.grad is None
        assert torch.equal(w.main_grad, ref.weight.grad)
        assert not w._mxk_grad_fresh and calls == [1]
        e(t).backward(g)                            # second micro-batch: added
        assert torch.equal(w.main_grad, ref.weight.grad + ref.weight.grad)
        assert calls == [1, 1]


def test_marked_direct_for_the_flat_buffer():
    assert Embedding(10, 4).weight._mxk_direct_grad
