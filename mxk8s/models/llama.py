"""Llama-3 architecture (random init) for the DDP validator / training bench.

BASELINE.json config 5: "PyTorch-ROCm DDP pod, Llama-3-8B synthetic training
step on amd.com/gpu=8".  The reference has no model code at all (SURVEY.md
§2.5); this is a from-scratch MI355X-first implementation:

* fused projections: one [q|k|v] GEMM per attention block and one [gate|up]
  GEMM per MLP (fewer, larger GEMMs), every product of the step on the
  hand-written MFMA kernels (``mxk8s.ops.linear``; SwiGLU fused into the
  [gate|up] epilogue);
* hand-written HIP kernels for the memory-bound glue: RMSNorm fwd/bwd,
  SwiGLU fwd/bwd, rotary embedding fwd/bwd (``mxk8s.ops.fused``);
* causal GQA attention through the hand-written gfx950 flash-attention
  kernels (``mxk8s.ops.attention``: forward + LSE, dQ and dK/dV passes) on
  q/k/v in their [B, S, H, D] projection layout (v stays a view of the fused
  QKV output); shapes those kernels do not tile fall back to SDPA;
* bf16 parameters; fp32 master weights and AdamW state live in the optimizer
  (``mxk8s.parallel.optim.FlatAdamW``).
"""
from __future__ import annotations

import dataclasses
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.attention import (flash_attention, proj_rope_attention, qkv_rope_attention,
                              supported as flash_supported)
from ..ops.linear import Linear, SwiGLULinear, swiglu_mlp
from ..ops.xent import cross_entropy
from ..ops.embedding import Embedding
from ..ops.fused import add_rmsnorm, qkv_rope, rmsnorm, rope_tables


@dataclasses.dataclass
class LlamaConfig:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    vocab_size: int = 128256
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq_len: int = 8192

    @classmethod
    def llama3_8b(cls) -> "LlamaConfig":
        return cls()

    @classmethod
    def tiny(cls) -> "LlamaConfig":
        # head_dim 128 like Llama-3, so the GPU tests run the HIP attention
        return cls(dim=512, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=1024, vocab_size=1024,
                   max_seq_len=512)

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def num_params(self) -> int:
        d, f, v, L = self.dim, self.ffn_dim, self.vocab_size, self.n_layers
        kv = self.n_kv_heads * self.head_dim
        per_layer = d * (d + 2 * kv) + d * d + 3 * d * f + 2 * d
        return L * per_layer + 2 * v * d + d

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token: 6 * params (matmuls) + attention (causal)."""
        n = self.num_params() - self.vocab_size * self.dim   # embedding lookup is free
        attn = 6 * self.n_layers * self.dim * seq_len       # 12*L*d*S, halved by causality
        return 6.0 * n + attn


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))
        # gradient straight into the flat buffer (mxk8s.ops.fused._deliver_dw);
        # MXK_DIRECT_NORM=1 (opt-in: step-neutral, profiles/r6_norm/)
        self.weight._mxk_direct_grad = os.environ.get("MXK_DIRECT_NORM", "0") == "1"

    def forward(self, x):
        return rmsnorm(x, self.weight, self.eps)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        hd = cfg.head_dim
        self.wqkv = Linear(cfg.dim, (cfg.n_heads + 2 * cfg.n_kv_heads) * hd)
        self.wo = Linear(cfg.n_heads * hd, cfg.dim)

    def forward(self, x, cos, sin):
        B, S, _ = x.shape
        c = self.cfg
        hd = c.head_dim
        # projection + RoPE (in the GEMM's epilogue) + flash attention as one
        # node; its backward takes d(qkv) from the attention kernels with the
        # RoPE backward fused into their stores
        o = proj_rope_attention(x, self.wqkv.weight, cos, sin, c.n_heads, c.n_kv_heads, hd)
        if o is not None:
            return self.wo(o.reshape(B, S, c.n_heads * hd))
        qkv = self.wqkv(x)
        # split + RoPE + flash attention as one node: its backward returns
        # d(qkv) with the RoPE backward fused into the attention kernels
        o = qkv_rope_attention(qkv, cos, sin, c.n_heads, c.n_kv_heads, hd)
        if o is not None:
            return self.wo(o.reshape(B, S, c.n_heads * hd))
        # q, k rotated straight out of their qkv slices; v a view into qkv
        # (token stride (Hq+2Hkv)*hd); one d(qkv) buffer in the backward
        q, k, v = qkv_rope(qkv, cos, sin, c.n_heads, c.n_kv_heads, hd)
        if flash_supported(q, k, v):
            # hand-written gfx950 flash attention: [B,S,H,D] in and out, no transposes
            o = flash_attention(q, k, v, causal=True)
            return self.wo(o.reshape(B, S, c.n_heads * hd))
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                           is_causal=True, enable_gqa=True)
        return self.wo(o.transpose(1, 2).reshape(B, S, c.n_heads * hd))


class MLP(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.w13 = Linear(cfg.dim, 2 * cfg.ffn_dim)   # [gate | up]
        # w2(swiglu(.)) as one node: the SwiGLU backward runs in the epilogue
        # of w2's input-gradient GEMM
        self.w2 = SwiGLULinear(cfg.ffn_dim, cfg.dim)

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.bfloat16:
            # one node: up-projection with SwiGLU in its epilogue, down
            # projection, fused dgrad-SwiGLU backward (mxk8s.ops.linear)
            return swiglu_mlp(x, self.w13.weight, self.w2.weight)
        return self.w2(self.w13(x))


class Block(nn.Module):
    """Pre-norm block.  ``forward(h, y)`` takes the residual stream h and its
    already-normalised copy y = attn_norm(h) and returns the block's output
    residual and the MLP delta still to be added, so every residual add is
    fused into the following RMSNorm (``add_rmsnorm``)."""

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.attn_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.attn = Attention(cfg)
        self.mlp_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.mlp = MLP(cfg)

    def forward(self, h, y, cos, sin):
        a = self.attn(y, cos, sin)
        h, y2 = add_rmsnorm(h, a, self.mlp_norm.weight, self.mlp_norm.eps)
        return h, self.mlp(y2)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        # the weight gradient straight into the flat buffer (mxk8s.ops.embedding);
        # MXK_DIRECT_EMBED=0: nn.Embedding + AccumulateGrad (A/B; same-box step
        # -1.1 / -1.3 ms, bit-identical losses: profiles/r6_embed/)
        direct = os.environ.get("MXK_DIRECT_EMBED", "1") != "0"
        self.embed = (Embedding if direct else nn.Embedding)(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layers)])
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.lm_head = Linear(cfg.dim, cfg.vocab_size)
        self._rope = {}   # device -> (cos, sin) fp32 tables, never cast with the model
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self, seed: int = 0) -> None:
        """Random init (N(0, 0.02), residual projections scaled by 1/sqrt(2L)),
        generated on the parameters' own device: an 8B model initialises in
        seconds on the GPU instead of minutes on the host."""
        gens = {}
        std = 0.02
        for name, p in self.named_parameters():
            if p.dim() == 1:
                p.fill_(1.0)
                continue
            if p.device not in gens:
                gens[p.device] = torch.Generator(device=p.device).manual_seed(seed)
            s = std / math.sqrt(2 * self.cfg.n_layers) if name.endswith(("wo.weight", "w2.weight")) else std
            p.normal_(0.0, s, generator=gens[p.device])

    def rope_tables(self, device) -> tuple[torch.Tensor, torch.Tensor]:
        key = str(device)
        if key not in self._rope:
            self._rope[key] = rope_tables(self.cfg.max_seq_len, self.cfg.head_dim,
                                          self.cfg.rope_theta, device=device)
        return self._rope[key]

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        cos, sin = self.rope_tables(tokens.device)
        h = self.embed(tokens)
        y = rmsnorm(h, self.layers[0].attn_norm.weight, self.cfg.norm_eps) if self.layers else h
        for i, layer in enumerate(self.layers):
            h, delta = layer(h, y, cos, sin)
            nxt = self.layers[i + 1].attn_norm if i + 1 < len(self.layers) else self.norm
            h, y = add_rmsnorm(h, delta, nxt.weight, nxt.eps)
        return self.lm_head(y)

    def loss(self, tokens: torch.Tensor, labels: torch.Tensor | None = None) -> torch.Tensor:
        """Next-token cross entropy (fp32 softmax)."""
        if labels is None:
            inp, labels = tokens[:, :-1], tokens[:, 1:]
        else:
            inp = tokens
        logits = self(inp)
        # fused bf16 softmax cross-entropy on GPU (no fp32 logits copy)
        return cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1))
