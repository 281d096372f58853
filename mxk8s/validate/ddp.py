"""Validator config 5 (Llama-3-8B DDP step) — see :mod:`mxk8s.train.ddp_llama`."""
from ..train.ddp_llama import run_ddp_bench  # noqa: F401
