"""GPU, world_size 2 and 8: utterance sharding end to end on the device. Two processes
(gloo group; both ranks drive cuda:0 here — the one-GPU box) get the weights by one broadcast of the
packed bf16 blob, decode their shard of the batch through libwcb with the bias boost, and gather the
ids; the concatenation in rank order equals the single-process decode of the whole batch. Cases:
tiny.en (6 clips, plumbing) and C4's model, whisper-small bf16, 2 ranks x 16 clips with the
1000-phrase boost (scripts/evaluation.py:173-206 decode contract on each shard)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

# name: (model, clips, tokens, bias phrases); "c4" = BASELINE config C4 at its stated shape: whisper-small,
# 256 clips over 8 ranks (32 per rank), 64 tokens with EOS masked, the 1000-phrase boost at lambda 2
CASES = {"tiny.en": ("tiny.en", 6, 16, 200), "small": ("small", 32, 16, 1000), "c4": ("small", 256, 64, 1000)}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _decode(model, lo, hi, dims, tokens, n_phr):
    from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list
    pcm = torch.from_numpy(synth_batch(hi - lo, start=lo)).cuda()
    mel = model.log_mel(pcm)
    phrases = synth_bias_list(n_phr, eot=dims.eos_token_id)
    ids = model.generate(mel, max_length=tokens, min_new_tokens=tokens, bias_list=phrases, bias_boost=2.0)
    return ids.cpu()


def _worker(rank, world, port, outdir, name):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from whisper_context_biasing_amd.config import get_dims
    from whisper_context_biasing_amd.model import WhisperCB
    from whisper_context_biasing_amd.shard import broadcast_weights, gather_shards, shard_bounds
    torch.cuda.set_device(0)
    size, n_clips, tokens, n_phr = CASES[name]
    dims = get_dims(size)
    sd = broadcast_weights(dims, torch.device("cpu"), seed=0)
    model = WhisperCB.from_state_dict(dims, sd, dtype="bf16")
    lo, hi = shard_bounds(n_clips, rank, world)
    ids = _decode(model, lo, hi, dims, tokens, n_phr)
    rows = torch.cat(gather_shards(ids, torch.device("cpu"), pad_value=dims.pad_token_id))
    if rank == 0:
        np.save(os.path.join(outdir, "sharded.npy"), rows.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_bench_launches_its_own_ranks(world):
    """`python bench.py --gpus N` with no torch.distributed.run: the launcher starts N ranks (gloo, all on
    this box's GPU), each decodes its 32 clips, rank 0 prints the whole-job line. N = 8 is the command form
    of the driver's C4 scaling run (8 x 32 = 256 clips, utterance-dp8)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    steps = 2 if world == 2 else 1
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "bench.py"), "--gpus", str(world), "--steps",
                        str(steps), "--warmup", "1", "--no-cpu-baseline", "--no-profile", "--backend", "gloo"],
                       capture_output=True, text=True, timeout=900, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [s for s in p.stdout.splitlines() if s.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["parallelism"] == f"utterance-dp{world}"
    assert out["config"]["global_batch"] == 32 * world and out["config"]["collective_backend"] == "gloo"
    assert out["value"] > 0 and out["steps"] == steps


@pytest.mark.parametrize("name,world", [("tiny.en", 2), ("small", 2), ("c4", 8)])
def test_rank_shards_equal_single_process(tmp_path, name, world):
    """world ranks (gloo, all on this box's one GPU) decode their shards; the ids gathered in rank order
    equal the single-process decode of the whole batch (generate() splits it into 64-clip calls). The
    ("c4", 8) case is C4's shape: 8 ranks x 32 clips = 256, whisper-small bf16, 64 tokens, 1000 phrases."""
    from whisper_context_biasing_amd.config import get_dims
    from whisper_context_biasing_amd.model import WhisperCB
    from whisper_context_biasing_amd.shard import broadcast_weights
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), name), nprocs=world, join=True)
    sharded = np.load(tmp_path / "sharded.npy")
    size, n_clips, tokens, n_phr = CASES[name]
    dims = get_dims(size)
    model = WhisperCB.from_state_dict(dims, broadcast_weights(dims, torch.device("cpu"), seed=0), dtype="bf16")
    full = _decode(model, 0, n_clips, dims, tokens, n_phr).numpy()
    assert sharded.shape == full.shape == (n_clips, tokens)
    np.testing.assert_array_equal(sharded, full)
