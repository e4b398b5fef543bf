"""Utterance sharding across ranks (one process per GPU).

The reference evaluates on one device (`scripts/evaluation.py:185-200`, `Seq2SeqTrainer`); clips
are independent, so N GPUs take disjoint shards of the utterance list and never exchange data on the
decode path. The only collectives are a one-time weight broadcast (RCCL over xGMI on the GPU box,
`gloo` in the CPU tests) and the max-over-ranks of the wall time in `bench.py`.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .config import WhisperDims
from .weights import make_weights, param_shapes


def shard_bounds(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of `n_items` for `rank` (sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    lo = n_items * rank // world
    hi = n_items * (rank + 1) // world
    return lo, hi


def pack_state_dict(dims: WhisperDims, sd: Dict[str, np.ndarray], dtype=torch.bfloat16) -> torch.Tensor:
    """All parameters in `param_shapes` order as one flat tensor (one collective moves them all)."""
    return torch.cat([torch.as_tensor(np.asarray(sd[n], dtype=np.float32)).reshape(-1)
                      for n, _ in param_shapes(dims)]).to(dtype)


def unpack_state_dict_views(dims: WhisperDims, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Views of every parameter into the packed blob, on the blob's device (no copy): on a GPU rank
    they feed wcb_load_weights directly."""
    out, off = {}, 0
    for n, shape in param_shapes(dims):
        k = int(np.prod(shape))
        out[n] = flat[off:off + k].view(*shape)
        off += k
    if off != flat.numel():
        raise ValueError(f"packed blob has {flat.numel()} elements, parameters need {off}")
    return out


def unpack_state_dict(dims: WhisperDims, flat: torch.Tensor) -> Dict[str, np.ndarray]:
    host = flat.float().cpu().numpy()
    out, off = {}, 0
    for n, shape in param_shapes(dims):
        k = int(np.prod(shape))
        out[n] = host[off:off + k].reshape(shape)
        off += k
    if off != host.size:
        raise ValueError(f"packed blob has {host.size} elements, parameters need {off}")
    return out


def broadcast_weights(dims: WhisperDims, device: torch.device, seed: int = 0, src: int = 0,
                      dtype=torch.bfloat16, views: bool = False) -> Dict[str, np.ndarray]:
    """Rank `src` materialises the seeded weights; one broadcast of the packed blob to every rank.
    Without an initialised process group this is just the local materialisation. `views`: return
    device views into the received blob (WhisperCB.load_state_dict hands them to wcb_load_weights
    without a host round trip) instead of host arrays."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    n_el = sum(int(np.prod(s)) for _, s in param_shapes(dims))
    # gloo moves host tensors: the blob crosses on the CPU and lands on `device` afterwards
    comm = _comm_device(device)
    if rank == src:
        flat = pack_state_dict(dims, make_weights(dims, seed=seed), dtype).to(comm)
    else:
        flat = torch.empty(n_el, dtype=dtype, device=comm)
    if world > 1:
        dist.broadcast(flat, src=src)
    flat = flat.to(device)
    return unpack_state_dict_views(dims, flat) if views else unpack_state_dict(dims, flat)


def _comm_device(device: torch.device) -> torch.device:
    """Where a collective's tensors must live: the rank's GPU under nccl (RCCL), the host under gloo."""
    if dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return torch.device(device)


def max_over_ranks(value: float, device: torch.device) -> float:
    """The slowest rank's time (bench.py reports whole-job throughput against it)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=_comm_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_shards(local: torch.Tensor, device: torch.device, pad_value: int) -> List[torch.Tensor]:
    """Collect every rank's result rows (evaluation-time convenience; not on the timed path).

    Ranks may return different numbers of rows and — with natural-EOS decoding, where generate()
    trims each shard to its own longest row — different widths: both are all-gathered first, every
    shard is padded (rows with zeros, columns with `pad_value` — the caller passes the model's pad
    id, WhisperDims.pad_token_id) to the global maximum for the collective, and each rank's rows come
    back at the common width. 1-D locals (one value per row) come back 1-D."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [local]
    world = dist.get_world_size()
    device = _comm_device(device)
    one_d = local.dim() == 1
    local = local.reshape(local.shape[0], -1) if one_d else local
    shp = torch.tensor([local.shape[0], local.shape[1] if local.dim() > 1 else 1], dtype=torch.int64, device=device)
    shps = [torch.zeros_like(shp) for _ in range(world)]
    dist.all_gather(shps, shp)
    mr = int(max(int(x[0].item()) for x in shps))
    mc = int(max(int(x[1].item()) for x in shps))
    buf = torch.full((mr, mc) + tuple(local.shape[2:]), pad_value, dtype=local.dtype, device=device)
    buf[local.shape[0]:] = 0
    buf[:local.shape[0], :local.shape[1]] = local.to(device)
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    out = [b[:int(k[0].item())] for b, k in zip(bufs, shps)]
    return [o[:, 0] for o in out] if one_d else out
