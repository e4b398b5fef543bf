"""CPU, world_size 2 over gloo: the multi-GPU path of bench.py (utterance sharding, one-time weight
broadcast, max-over-ranks timing, result gather) without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from whisper_context_biasing_amd.config import get_dims
from whisper_context_biasing_amd.shard import (broadcast_weights, gather_shards, max_over_ranks,
                                               pack_state_dict, shard_bounds, unpack_state_dict)
from whisper_context_biasing_amd.synth import synth_batch
from whisper_context_biasing_amd.weights import make_weights


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    dims = get_dims("micro")
    sd = broadcast_weights(dims, dev, seed=3)
    per_rank = 3
    lo, hi = shard_bounds(world * per_rank, rank, world)
    pcm = synth_batch(hi - lo, start=lo, n_samples=1600)
    t = max_over_ranks(0.25 * (rank + 1), dev)
    ids = torch.arange(lo, hi, dtype=torch.int64)[:, None] * 10 + torch.arange(4)
    rows = torch.cat(gather_shards(ids, dev, pad_value=50257))
    flat = torch.cat(gather_shards(ids[:, 0], dev, pad_value=50257))   # 1-D locals stay 1-D
    # natural-EOS decoding trims each shard to its own longest row: unequal widths (and row counts)
    wide = torch.arange(lo, hi, dtype=torch.int64)[:, None] * 10 + torch.arange(3 + 2 * rank)
    ragged = torch.cat(gather_shards(wide if rank == 0 else wide[:2], dev, pad_value=50257))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), pcm=pcm, t=t, rows=rows.numpy(), flat=flat.numpy(), lo=lo, hi=hi, ragged=ragged.numpy(),
             **{f"w_{k.replace('.', '_')}": v for k, v in sd.items() if "layers.0" in k or "embed" in k})
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_partition():
    for n in (0, 1, 7, 64, 256):
        for world in (1, 2, 3, 8):
            parts = [shard_bounds(n, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            sizes = [hi - lo for lo, hi in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(8, 2, 2)


def test_pack_unpack_roundtrip():
    dims = get_dims("micro")
    sd = make_weights(dims, seed=1)
    back = unpack_state_dict(dims, pack_state_dict(dims, sd, torch.float32))
    assert set(back) == set(sd)
    for k in sd:
        np.testing.assert_array_equal(back[k], sd[k].astype(np.float32))


def test_two_rank_gloo(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{i}.npz") for i in range(world)]
    # disjoint shards that together are exactly the single-process batch
    assert (r[0]["lo"], r[0]["hi"], r[1]["lo"], r[1]["hi"]) == (0, 3, 3, 6)
    np.testing.assert_array_equal(np.concatenate([r[0]["pcm"], r[1]["pcm"]]), synth_batch(6, n_samples=1600))
    # the slowest rank's time
    assert float(r[0]["t"]) == float(r[1]["t"]) == 0.5
    # every rank gathered all rows in rank order
    for x in r:
        np.testing.assert_array_equal(x["rows"][:, 0], np.arange(6) * 10)
        assert x["flat"].shape == (6,)
        np.testing.assert_array_equal(x["flat"], np.arange(6) * 10)
        # ragged shards: rank 0 sent 3 rows x 3 columns, rank 1 2 rows x 5 columns; every rank holds
        # 5 rows at width 5, rank 0's rows right-padded with the pad id
        rg = x["ragged"]
        assert rg.shape == (5, 5)
        np.testing.assert_array_equal(rg[:3, :3], np.arange(3)[:, None] * 10 + np.arange(3))
        assert (rg[:3, 3:] == 50257).all()
        np.testing.assert_array_equal(rg[3:], np.arange(3, 5)[:, None] * 10 + np.arange(5))
    # rank 1 received rank 0's weights bit-for-bit (bf16 blob), equal to the seeded weights
    ref = make_weights(get_dims("micro"), seed=3)
    keys = [k for k in r[0].files if k.startswith("w_")]
    assert keys
    for k in keys:
        np.testing.assert_array_equal(r[0][k], r[1][k])
    k0 = "model.decoder.embed_tokens.weight"
    want = torch.from_numpy(ref[k0]).to(torch.bfloat16).float().numpy()
    np.testing.assert_array_equal(r[1]["w_" + k0.replace(".", "_")], want)
