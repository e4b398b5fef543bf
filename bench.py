#!/usr/bin/env python3
"""Benchmark of the Whisper contextual-biasing hot path on MI355X (BASELINE.json metric).

One "step" = the full inference path for one batch of synthetic 30 s / 16 kHz clips already
resident in HBM: log-mel → encoder → greedy decode of exactly 64 new tokens (EOS masked,
SURVEY.md §8(d) benchmark mode) with the fused bias-list boost (1000 phrases, lambda 2.0).
Default workload = config C2: whisper-small, batch 32 per GPU, bf16 (random-init weights of that
architecture; no checkpoint offline).

Multi-GPU: one process per GPU, utterances sharded (weak scaling: 32 clips per GPU), weights
generated on rank 0 and broadcast once over RCCL/xGMI (`dist.broadcast`), no collective in the
timed region besides the barriers; time = max over ranks. Two ways in:
  * `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` (WORLD_SIZE set: this
    process is one rank);
  * `python bench.py --gpus N` (WORLD_SIZE unset): this process is only a launcher — it starts N
    rank processes of itself before anything touches the GPU (it never initialises HIP), forwards
    rank 0's JSON line and exits non-zero when any rank fails (the others are then stopped).
`--backend nccl` (default: RCCL, rank r on GPU r) or `gloo` (ranks may share a GPU: rank r on GPU
r mod the device count — how the N>1 path is exercised on a one-GPU box).

Prints ONE JSON line (rank 0) with the driver's contract fields plus `roofline` (dominant kernel:
the kernel symbol with the most device time per step, grouped as rocprofv3 --stats groups them, from
begin/end timestamps of every launch in a serialised profiling pass; at C2 that is the decode's
encoder-space cross-attention, whose per-launch time is then taken from device stamps in its
decode-graph nodes in a pass pipelined exactly as the timed region) and
`cpu_baseline` (the fp32 PyTorch-CPU restatement, both reference decode modes, timed on this host,
rank 0 / N=1 only).

`--reference-mode`: the reference's own decode contract instead of the benchmark mode —
natural EOS, max_length=225, no boost (scripts/evaluation.py:173-179), same clips; its line goes to
profiles/ beside the benchmark line (not the driver's headline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table)
PEAK_F16_TFLOPS = 2500.0
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0
ENC_GEMMS = ("enc_conv1", "enc_conv2", "enc_qkv", "enc_out", "enc_fc1", "enc_fc2")
DEC_PROJ = ("dec_qkv", "dec_out", "dec_xq", "dec_kq", "dec_vg", "dec_xo", "dec_fc1", "dec_fc2", "lm_head")


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share():
    """CPUs this process may actually use: the affinity mask and the cgroup v2/v1 CPU quota (the GPU
    box gives each job a share of a large host: os.cpu_count() counts the whole host)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    share = aff if quota is None else max(1, min(aff, int(quota)))
    return share, aff, quota


def cpu_baseline(size: str, n_tokens: int, n_phr: int, boost: float, seed: int = 0, clips: int = 1, reps: int = 10,
                 warmups: int = 3):
    """the fp32 PyTorch-CPU restatement of the reference path (oracle/whisper_torch.py,
    test infrastructure) on this host's CPU share (affinity mask / cgroup quota; os.cpu_count() counts
    the whole host), on a bounded sample of the same workload — `clips` clip(s) per run: log-mel +
    encoder + n_tokens greedy tokens with the same bias list and boost — in the reference's two decode
    modes: (i) use_cache=False exactly as scripts/evaluation.py:178 configures generate(), (ii)
    KV-cached. `warmups` untimed runs (three), then the median of `reps` (>= 10) timed
    runs per mode (the runs of the two modes interleaved). `value` = mode (ii), the faster one. Nothing is extrapolated: the sample
    is `clips` clip(s) per run, not the 32-clip batch."""
    import torch
    from oracle import whisper_torch as WT
    from whisper_context_biasing_amd.config import get_dims
    from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list, synth_word_start
    from whisper_context_biasing_amd.weights import make_weights
    share, aff, quota = _cpu_share()
    torch.set_num_threads(share)
    dims = get_dims(size)
    m = WT.TorchWhisper(dims, make_weights(dims, seed=seed))
    pcm = torch.from_numpy(synth_batch(clips))
    phrases = synth_bias_list(n_phr, eot=dims.eos_token_id)
    kw = dict(min_new_tokens=n_tokens, bias=phrases, bias_boost=boost,
              word_start=synth_word_start(dims.eos_token_id, dims.vocab))

    def run(use_cache, tokens=n_tokens):
        t0 = time.perf_counter()
        mel = WT.log_mel(pcm, dims.n_mel)
        m.generate(mel, use_cache=use_cache, max_length=tokens, **dict(kw, min_new_tokens=tokens))
        return time.perf_counter() - t0

    with torch.no_grad():
        for i in range(warmups):                      # thread pool, allocator, page-in (short runs)
            run(i % 2 == 0, tokens=4)
        t_c, t_n = [], []
        for _ in range(reps):
            t_c.append(run(True))
            t_n.append(run(False))
    t_cached, t_nocache = float(np.median(t_c)), float(np.median(t_n))
    return {"value": round(clips * 30.0 / t_cached, 3), "unit": "audio-seconds/sec",
            "cores": torch.get_num_threads(), "kind": "port",
            "cpu_share": {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "threads_used": torch.get_num_threads(),
                          "host_cpu_count": os.cpu_count(), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")},
            "cpu_model": _cpu_model(),
            "modes": {"kv_cached": round(clips * 30.0 / t_cached, 3),
                      "use_cache_false_reference_config": round(clips * 30.0 / t_nocache, 3)},
            "runs_s": {"kv_cached": [round(t, 3) for t in t_c], "use_cache_false": [round(t, 3) for t in t_n]},
            "sample": f"{clips} clip(s) x 30 s per run, whisper-{size} fp32 PyTorch-CPU restatement of the reference "
                      f"path (oracle/whisper_torch.py): log-mel + encoder + {n_tokens} greedy tokens with the "
                      f"{n_phr}-phrase boost; {warmups} warm-ups, median of {reps} runs per mode: kv-cached "
                      f"{t_cached:.2f} s, use_cache=False (scripts/evaluation.py:178) {t_nocache:.2f} s wall; "
                      f"{torch.get_num_threads()} threads = this job's CPU share (affinity {aff}, cgroup quota "
                      f"{quota}); not extrapolated to the 32-clip batch"}


# phase of every profiled launch class (bench `phases` keys / rocprofv3 kernel symbols via tools/check_roofline.py)
FRONT_CLASSES = ("log_mel", "mel_to_conv_input")


def _phase_of(cls: str) -> str:
    if cls in FRONT_CLASSES:
        return "front_end"
    if cls.startswith("enc_") or cls == "layernorm":
        return "encoder"
    return "decode"


def step_ideal(dims, clips: int, new_tokens: int, num_beams: int = 1, esize: int = 2,
               peak_mfma_tflops: float = PEAK_BF16_TFLOPS, peak_hbm_gbs: float = PEAK_HBM_GBS, prompt_len: int = 1):
    """SURVEY §8(d)'s step roofline: each phase's ideal time at its roofline, from algorithmic work alone
    (no kernel's own accounting). front end (HBM): PCM in + mel out, f32. encoder (MFMA): conv stem + layer
    GEMMs (2·M·N·K) + attention (4·S²·d per layer). decode (HBM), per generated token: every decoder weight
    once (16·d² per layer + the tied V·d LM head) + the cross-attention's encoder-side bytes at the fewest
    any formulation needs (the encoder output once per clip per layer: the encoder-space algebra; the K/V
    form reads twice that) + the self-attention K/V cache of every row at its position (keys 1 .. t).
    Returns {phase: ideal ms per step} and the bytes / flops behind them."""
    d, L, S, V, nm = dims.d_model, dims.n_layers, dims.n_audio_ctx, dims.vocab, dims.n_mel
    frames = 2 * S
    front_bytes = clips * (480000 * 4 + nm * frames * 4)
    enc_flops = clips * (2.0 * frames * d * 3 * nm + 2.0 * S * d * 3 * d
                         + L * (2.0 * S * 12 * d * d + 4.0 * S * S * d))
    rows = clips * num_beams
    w_bytes = (L * 16 * d * d + V * d) * esize
    x_bytes = clips * L * S * d * esize                       # per token
    kv_bytes = sum(rows * 2 * L * (prompt_len - 1 + t) * d * esize for t in range(1, new_tokens + 1))
    dec_bytes = new_tokens * (w_bytes + x_bytes) + kv_bytes
    ideal = {"front_end": front_bytes / (peak_hbm_gbs * 1e9) * 1e3,
             "encoder": enc_flops / (peak_mfma_tflops * 1e12) * 1e3,
             "decode": dec_bytes / (peak_hbm_gbs * 1e9) * 1e3}
    return ideal, {"front_end_bytes": front_bytes, "encoder_flops": enc_flops, "decode_bytes": dec_bytes,
                   "decode_bytes_per_token": {"weights": w_bytes, "encoder_side": x_bytes,
                                              "self_kv_mean": kv_bytes / max(new_tokens, 1)}}


def step_roofline(dims, clips, new_tokens, num_beams, esize, peak_mfma, ms_per_step, phases):
    """roofline.step: Σ(phase ideal time) ÷ the measured step time (the timed region's, pipelined), and per
    phase its ideal time ÷ its serialised GPU time from the profiling pass (`phases`)."""
    ideal, work = step_ideal(dims, clips, new_tokens, num_beams, esize, peak_mfma)
    meas = {}
    for k, v in (phases or {}).items():
        if k.startswith("family:"):
            continue
        ph = _phase_of(k)
        meas[ph] = meas.get(ph, 0.0) + v["ms_per_step"]
    tot = sum(ideal.values())
    per = {ph: {"ideal_ms": round(ideal[ph], 4), "bound": "mfma" if ph == "encoder" else "hbm",
                "serialised_ms": round(meas[ph], 3) if ph in meas else None,
                "frac": round(ideal[ph] / meas[ph], 4) if meas.get(ph) else None} for ph in ideal}
    return {"ideal_ms": round(tot, 4), "measured_ms_per_step": round(ms_per_step, 3),
            "frac": round(tot / ms_per_step, 4), "phases": per,
            "serialised_gpu_ms": round(sum(meas.values()), 3) if meas else None,
            "work": {k: (round(v, 1) if isinstance(v, float) else v) for k, v in work.items()},
            "definition": "SURVEY §8(d): frac = Σ(phase ideal time at its roofline) ÷ measured ms_per_step; encoder "
                          "FLOPs at the dense MFMA peak, front end and decode bytes at 8 TB/s (decode: decoder "
                          "weights + the encoder output once per clip per layer + self-K/V, per token); phase frac = "
                          "ideal ÷ that phase's serialised GPU time (profiling pass)"}


def _pmc_traffic(kernel: str, grid=None):
    """HBM bytes per launch of `kernel` (symbol, every grid it runs at) from the committed rocprofv3
    PMC passes (profiles/*pmc*.json, written by tools/pmc_traffic.py: FETCH_SIZE x 2 (gfx950
    correction) + WRITE_SIZE), or None."""
    import glob
    # profiles/ stays on the build host (.gpurunignore); the latest PMC summary also ships as
    # tools/pmc_traffic_latest.json (a copy of the newest profiles/*pmc_traffic.json)
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True)
    paths.append(os.path.join(ROOT, "tools", "pmc_traffic_latest.json"))
    for path in paths:
        if not os.path.exists(path):
            continue
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        # the launch shape's own figure first (one symbol runs at several grids: prefill, beams)
        e = d.get("kernels", {}).get(f"{kernel}|{grid}") if grid else None
        e = e or d.get("symbols", {}).get(kernel)
        if e:
            return e["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None


def _config_tag(args, world):
    """BASELINE.json configs: C2 small/32/greedy, C3 medium/64/beam-5, C4 small sharded, C5 large-v3/16/beam-5."""
    if args.num_beams > 1:
        return {"medium": "C3", "large-v3": "C5"}.get(args.model, "beam")
    return ("C4" if world > 1 else "C2") if args.model == "small" else "greedy"


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(cmd, n, env_extra=None, grace_s=15.0, poll_s=0.2):
    """Run `n` rank processes of `cmd` (one per GPU) and wait for them. Each gets RANK / LOCAL_RANK /
    WORLD_SIZE / LOCAL_WORLD_SIZE and a 127.0.0.1 rendezvous (MASTER_ADDR / MASTER_PORT), as
    torch.distributed.run would set them. Rank 0's stdout is forwarded line by line and its last
    JSON line kept; the other ranks inherit stdout / stderr. When a rank exits non-zero the others
    are terminated (SIGTERM, SIGKILL after `grace_s`) — by the PIDs started here, never by pattern.
    Returns (exit code, rank 0's last JSON line or None): 0 only when every rank exited 0 and rank 0
    printed a JSON line. This process starts no GPU work of its own."""
    import subprocess
    import threading
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), **(env_extra or {}))
    procs, last_json = [], [None]
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else None, text=True))

    def pump():   # rank 0's stdout → ours
        for line in procs[0].stdout:
            sys.stdout.write(line)
            sys.stdout.flush()
            s = line.strip()
            if s.startswith("{") and s.endswith("}"):
                last_json[0] = s
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            log(f"launcher: a rank exited with {rc}; stopping the others")
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            t_end = time.time() + grace_s
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, t_end - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(poll_s)
    th.join(timeout=5.0)
    if rc == 0 and last_json[0] is None:
        log("launcher: rank 0 printed no JSON line")
        rc = 1
    return (rc if rc >= 0 else 128 - rc), last_json[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process group for N > 1 ranks: nccl (RCCL over xGMI, one GPU per rank) or gloo "
                         "(ranks may share a GPU: rank r on GPU r mod the device count)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="small")
    ap.add_argument("--batch", type=int, default=32, help="clips per GPU")
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--num-beams", type=int, default=1,
                    help="1 = greedy (C2/C4); 5 = the C3 / C5 beam configurations")
    ap.add_argument("--bias-phrases", type=int, default=1000)
    ap.add_argument("--boost", type=float, default=2.0)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=2, help="steps of the serialised roofline pass")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="wcb_set_option on the handle (alternative formulations, for sweeps)")
    ap.add_argument("--reference-mode", action="store_true",
                    help="the reference's decode contract: natural EOS, max_length=225, no boost "
                         "(scripts/evaluation.py:173-179); batches serialised (the host polls EOS)")
    ap.add_argument("--side-stream", action="store_true",
                    help="issue the step from a non-default torch stream (CU-masked library streams, option "
                         "cu_split, are blocking streams: work on the legacy null stream serialises them)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="serialise batches (default: batch i+1's front end + encoder overlap batch i's decode)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launcher: N fresh rank processes of this script, started before anything here touches the GPU
        rc, _ = launch_ranks([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], args.gpus)
        sys.exit(rc)
    if args.reference_mode:
        args.new_tokens, args.boost, args.no_overlap, args.no_cpu_baseline = 225, 0.0, True, True
    min_new = 0 if args.reference_mode else args.new_tokens   # benchmark mode: EOS masked, fixed length

    import torch
    import torch.distributed as dist
    from whisper_context_biasing_amd.config import get_dims
    from whisper_context_biasing_amd.model import WhisperCB
    from whisper_context_biasing_amd.synth import runner_up_phrases, synth_batch, synth_bias_list, synth_word_start
    from whisper_context_biasing_amd.shard import broadcast_weights, max_over_ranks, shard_bounds

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible")
    if args.backend == "nccl" and world > 1 and local >= ndev:
        raise SystemExit(f"bench.py: rank {rank} (local {local}) needs GPU {local} but {ndev} are visible; "
                         f"nccl takes one GPU per rank (--backend gloo lets ranks share one)")
    gpu = local % ndev
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if args.side_stream:
        torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    devices_used = min(world, ndev)

    dims = get_dims(args.model)
    # ---- weights: rank 0 generates, one RCCL broadcast of the packed bf16 blob over xGMI
    t0 = time.perf_counter()
    sd = broadcast_weights(dims, dev, seed=0, views=True)   # device views: no host round trip
    if world > 1:
        torch.cuda.synchronize()
        log(f"rank {rank}: weights broadcast in {time.perf_counter() - t0:.3f} s")
    opts = {k: int(v) for k, v in (o.split("=", 1) for o in args.opt)}
    model = WhisperCB.from_state_dict(dims, sd, dtype=args.dtype, device=gpu, options=opts or None)
    del sd

    B = args.batch
    lo, hi = shard_bounds(world * B, rank, world)                      # this rank's utterances
    pcm = torch.from_numpy(synth_batch(hi - lo, start=lo)).to(dev)     # resident in HBM before timing
    # bias list (untimed setup): matches start only at word-start tokens (synthetic half of the
    # vocabulary, the role of BPE's leading-space tokens); the reference's bias-word pool, plus one phrase
    # per clip built from its own lam = 0 decode's runner-up continuation at a step where a boost of
    # lam_plumb places it (so the biased-WER half of the metric measures the boost). lam_plumb is sized
    # to this random-weight model's logit gaps (2 x the median top-1/top-2 gap): the bench's lam = 2
    # is 10-30x those gaps and flips the first step of every clip (reported as measured, below).
    ws = synth_word_start(dims.eos_token_id, dims.vocab)
    model.set_word_start(ws)
    pool_all = synth_bias_list(args.bias_phrases, eot=dims.eos_token_id)
    targets, placed, lam_plumb, gaps = [], [], None, None
    if args.boost > 0 and args.num_beams == 1:
        mel0 = model.log_mel(pcm)
        _, _, _, gaps = runner_up_phrases(model, mel0, args.new_tokens, args.boost, ws)
        lam_plumb = round(2.0 * float(np.median(gaps[:, 1:])), 4)
        pool_cut = pool_all[:max(0, args.bias_phrases - B)]
        _, placed, targets, _ = runner_up_phrases(model, mel0, args.new_tokens, lam_plumb, ws, pool=pool_cut)
    seen = {tuple(p) for p in placed}
    pool = [p for p in pool_all if tuple(p) not in seen]
    phrases = placed + pool[:max(0, args.bias_phrases - len(placed))]
    bias = model.bias_list(phrases)
    use_graph = not args.no_graph

    overlap = not args.no_overlap
    keep = []   # async mode: inputs/outputs stay alive until the final synchronize

    def step():
        mel = model.log_mel(pcm)
        ids = model.generate(mel, max_length=args.new_tokens, min_new_tokens=min_new,
                             bias_list=phrases, bias_boost=args.boost, use_graph=use_graph, block=not overlap,
                             num_beams=args.num_beams)
        keep.append((mel, ids))
        return ids

    for i in range(args.warmup):
        ids = step()
        model.synchronize()
        torch.cuda.synchronize()
        log(f"warmup {i} done, ids {tuple(ids.shape)}")
    assert ids.shape[0] == B and (args.num_beams > 1 or min_new == 0 or ids.shape == (B, args.new_tokens))
    keep.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gen_tokens = 0
    for i in range(args.steps):
        ids = step()
        if not overlap:
            gen_tokens += int((ids != dims.pad_token_id).sum()) + int(ids.shape[0])   # + the final EOS of each row
    model.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * 30.0 / (elapsed / args.steps)
    keep.clear()

    # ---- per-kernel-class roofline: a separate, untimed pass of the same step in which every launch
    #      (front end, encoder, each decode-step kernel) carries the kernel's own begin/end timestamps
    #      (hipExtLaunchKernel events; the decode runs eagerly since a replayed graph node cannot carry
    #      them) — the source rocprofv3's kernel trace reads, so profiles/ reproduces these durations.
    prof, prof_steps = {}, 0
    if not args.no_profile:
        prof_steps = max(1, min(args.steps, args.profile_steps))
        model.profile_enable(True, events=True, stamps=False)
        for i in range(prof_steps):
            mel = model.log_mel(pcm)
            model.generate(mel, max_length=args.new_tokens, min_new_tokens=min_new, bias_list=phrases,
                           bias_boost=args.boost, use_graph=False, block=True, num_beams=args.num_beams)
        model.synchronize()
        torch.cuda.synchronize()
        prof = model.profile_read()
        model.profile_enable(False)
        prof.pop("decode_loop", None)
        prof.pop("xkv_gemm_total", None)
    # the dominant decode kernel (the encoder-space cross-attention, a node of the replayed decode graph)
    # timed again under the timed region's own conditions — graphs, batches in flight, the encoder of
    # the next batch beside it — from device stamps in its graph nodes (HIP events cannot bracket a
    # graph node): the per-launch time rocprofv3 sees over the same command
    xattn_live, graph_us = None, {}
    if not args.no_profile and args.num_beams == 1 and use_graph:
        model.profile_enable(True, events=False, stamps=True)
        for i in range(max(2, prof_steps)):
            step()
        model.synchronize()
        torch.cuda.synchronize()
        live = model.profile_read()
        e = live.get("dec_xattn")
        model.profile_enable(False)
        keep.clear()
        if e and e["launches"] and e["ms"] > 0:
            xattn_live = {"avg_ms": e["ms"] / e["launches"], "launches": e["launches"], "bytes": e["bytes"] / e["launches"]}
        # the lean decode projections stamped the same way (first workgroup start to last workgroup end of
        # each launch inside the replayed graph, both decode chains and the encoder in flight)
        graph_us = {k.split("@")[0]: round(v["ms"] / v["launches"] * 1e3, 3)
                    for k, v in live.items() if k.endswith("@graph") and v["launches"]}
    roof, others = None, {}
    if prof:
        peak_mfma = {"bf16": PEAK_BF16_TFLOPS, "f16": PEAK_F16_TFLOPS}.get(args.dtype, PEAK_F32_TFLOPS)
        classes = {}
        for k, v in prof.items():
            if not v["launches"] or v["ms"] <= 0:
                continue
            avg_ms = v["ms"] / v["launches"]
            mfma = k.startswith("enc_") or k == "xkv_gemm"   # encoder / cross-K/V GEMMs and flash attention
            if mfma:
                ach = v["flops"] / v["launches"] / (avg_ms * 1e-3) / 1e12
                peak, unit = peak_mfma, "TFLOP/s"
            else:
                ach = v["bytes"] / v["launches"] / (avg_ms * 1e-3) / 1e9
                peak, unit = PEAK_HBM_GBS, "GB/s"
            classes[k] = {"bound": "mfma" if mfma else "hbm",
                          "kernel": v.get("kernel", "").split("(")[0], "grid": v.get("grid", 0),
                          "achieved": round(ach, 1), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
                          "traffic": None, "avg_launch_ms": round(avg_ms, 5),
                          "launches_per_step": v["launches"] / prof_steps,
                          "bytes_per_launch": v["bytes"] / v["launches"], "flops_per_launch": v["flops"] / v["launches"],
                          "total_ms_per_step": round(v["ms"] / prof_steps, 3)}
        # dominant = the kernel symbol with the most time per step — rocprofv3 --stats' grouping, so the
        # classes one kernel instance serves (e.g. dec_qkv / dec_xq / dec_fc1) are summed as it sums them
        groups = {}
        for k, c in classes.items():
            gk = c["kernel"]
            g = groups.setdefault(gk, {"classes": [], "ms": 0.0, "launches": 0.0, "bytes": 0.0, "flops": 0.0})
            g["classes"].append(k)
            g["ms"] += c["total_ms_per_step"]
            g["launches"] += c["launches_per_step"]
            g["bytes"] += c["bytes_per_launch"] * c["launches_per_step"]
            g["flops"] += c["flops_per_launch"] * c["launches_per_step"]
        gk = max(groups, key=lambda k: groups[k]["ms"])
        g = groups[gk]
        dom = max(g["classes"], key=lambda k: classes[k]["total_ms_per_step"])
        c = classes[dom]
        avg_ms = g["ms"] / g["launches"]
        per = (g["flops"] if c["bound"] == "mfma" else g["bytes"]) / g["launches"]
        ach = per / (avg_ms * 1e-3) / (1e12 if c["bound"] == "mfma" else 1e9)
        dom_grid = c["grid"] if len(g["classes"]) == 1 else None
        roof = dict(c, **{"class": "+".join(sorted(g["classes"])), "achieved": round(ach, 1), "grid": dom_grid,
                          "frac": round(ach / c["peak"], 4), "avg_launch_ms": round(avg_ms, 5),
                          "launches_per_step": g["launches"], "bytes_per_launch": g["bytes"] / g["launches"],
                          "flops_per_launch": g["flops"] / g["launches"], "total_ms_per_step": round(g["ms"], 3),
                          "timing": "kernel begin/end timestamps of every launch (hipExtLaunchKernel events) in a "
                                    f"serialised profiling pass of {prof_steps} step(s); rocprofv3 trace of the "
                                    "same command: profiles/ (tools/check_roofline.py compares the two)"})
        if xattn_live and "dec_xattn" in g["classes"] and len(g["classes"]) == 1:
            # per-launch time under the timed region's conditions (device stamps, graphs, overlap); the
            # serialised profiling pass's value is kept beside it
            ach_live = roof["bytes_per_launch"] / (xattn_live["avg_ms"] * 1e-3) / 1e9
            roof.update({"avg_launch_ms_serialised": roof["avg_launch_ms"], "frac_serialised": roof["frac"],
                         "avg_launch_ms": round(xattn_live["avg_ms"], 5), "achieved": round(ach_live, 1),
                         "frac": round(ach_live / roof["peak"], 4),
                         "timing": f"device stamps (s_memrealtime, first workgroup start to last workgroup end) in "
                                   f"the decode-graph nodes of {xattn_live['launches']} launches, pipelined exactly as "
                                   "the timed region (graphs, batches in flight); avg_launch_ms_serialised = kernel "
                                   "begin/end HIP events of a serialised eager pass; rocprofv3 trace of the same "
                                   "command: profiles/ (tools/check_roofline.py compares the two)"})
        c2 = (args.model, args.batch, args.num_beams, args.dtype, args.new_tokens) == ("small", 32, 1, "bf16", 64)
        tr = _pmc_traffic(roof["kernel"], dom_grid) if c2 else None
        if tr:
            roof["traffic"], roof["traffic_source"] = tr
        others = {k: v for k, v in classes.items() if k not in g["classes"]}
    phases = {k: {"ms_per_step": round(v["ms"] / prof_steps, 3), "launches_per_step": v["launches"] / prof_steps}
              for k, v in prof.items()}
    if phases:   # family totals: every encoder GEMM, every decode projection (LM head included)
        fam = lambda pred: round(sum(v["ms_per_step"] for k, v in phases.items() if pred(k)), 3)
        phases["family:enc_gemm"] = {"ms_per_step": fam(lambda k: k in ENC_GEMMS)}
        phases["family:dec_proj"] = {"ms_per_step": fam(lambda k: k in DEC_PROJ)}
    esize = {"f32": 4, "fp32": 4}.get(args.dtype, 2)
    peak_mfma = {"bf16": PEAK_BF16_TFLOPS, "f16": PEAK_F16_TFLOPS, "fp16": PEAK_F16_TFLOPS}.get(args.dtype, PEAK_F32_TFLOPS)
    step_roof = step_roofline(dims, B, args.new_tokens, args.num_beams, esize, peak_mfma, ms_per_step, phases)
    if roof is not None:
        roof["step"] = step_roof

    # biased-WER half of the metric (random weights: no transcript to score against): the boosted
    # decode of the benchmark batch against its lam = 0 decode, scored by the C++ host scorer with
    # token ids as words — WER, compute_bias_wer's tallies over the bias list, and the recall of the
    # placed phrases (each clip's runner-up continuation, absent from its lam = 0 decode); untimed
    bias_plumb = None
    if rank == 0 and args.boost > 0:
        import ctypes as C
        from whisper_context_biasing_amd import _lib
        from whisper_context_biasing_amd.metrics import _cstrs, wer_counts
        mel = model.log_mel(pcm)
        kw = dict(max_length=args.new_tokens, min_new_tokens=min_new, use_graph=use_graph, num_beams=args.num_beams)
        plain = model.generate(mel, **kw).cpu().tolist()
        as_text = lambda rows: [" ".join(map(str, r)) for r in rows]
        ptxt = [" ".join(map(str, p)) for p in phrases]

        def score(lam):
            boosted = model.generate(mel, bias_list=phrases, bias_boost=lam, **kw).cpu().tolist()
            model.synchronize()
            err, words = wer_counts(as_text(boosted), as_text(plain))
            bd = bt = 0
            for r, h in zip(as_text(boosted), as_text(plain)):   # the list's phrases: boosted vs lam = 0
                d_, t_ = C.c_int64(), C.c_int64()
                _lib.check(_lib.load().wcb_bias_counts((" " + r + " ").encode(), (" " + h + " ").encode(),
                                                       _cstrs([" " + t + " " for t in ptxt]), len(ptxt),
                                                       C.byref(d_), C.byref(t_)), None, "wcb_bias_counts")
                bd += d_.value
                bt += t_.value
            has = lambda row, p: any(row[i:i + len(p)] == p for i in range(len(row) - len(p) + 1))
            n = len(placed)
            first_div = [next((i for i, (a, b) in enumerate(zip(x, y)) if a != b), len(x)) for x, y in zip(boosted, plain)]
            return {"lambda": lam,
                    "wer_boosted_vs_unboosted": round(100.0 * sum(err) / max(sum(words), 1), 3),
                    "bias_wer_unboosted_vs_boosted": round(100.0 * bd / bt, 3) if bt else 0.0,
                    "bias_phrase_tokens_in_boosted": bt,
                    "median_first_divergence_step": float(np.median(first_div)),
                    "placed_phrase_recall_boosted":
                        round(sum(has(boosted[b], placed[i]) for i, (b, _) in enumerate(targets)) / n, 4) if n else None,
                    "placed_phrase_recall_unboosted":
                        round(sum(has(plain[b], placed[i]) for i, (b, _) in enumerate(targets)) / n, 4) if n else None,
                    "placed_at_target_step_boosted":
                        round(sum(boosted[b][t:t + 2] == placed[i] for i, (b, t) in enumerate(targets)) / n, 4) if n else None,
                    "placed_at_target_step_unboosted":
                        round(sum(plain[b][t:t + 2] == placed[i] for i, (b, t) in enumerate(targets)) / n, 4) if n else None}

        bias_plumb = {"placed_phrases": len(placed), "bench_lambda": score(args.boost),
                      "plumb_lambda": score(lam_plumb) if lam_plumb else None,
                      "model_gap_quantiles_5_50_95": ([round(float(q), 4) for q in np.quantile(gaps[:, 1:], [0.05, 0.5, 0.95])]
                                                      if gaps is not None else None),
                      "note": "random weights: token ids as words. WER of the boosted decode against the lam=0 decode; "
                              "bias-WER of the lam=0 decode against the boosted one over the whole bias list; recall "
                              "of each clip's placed phrase (its lam=0 runner-up continuation at the earliest step "
                              "whose gap lies in [0.25, 0.75) x plumb_lambda, before the pool-only boosted decode "
                              "first diverges). The bench's lambda=2 exceeds this random model's top-1/top-2 gaps "
                              "(quantiles above), so it flips the first steps of every clip; plumb_lambda = 2 x the "
                              "median gap is the scale at which targeted placement is measurable."}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing the CPU oracle baseline ...")
        cpu = cpu_baseline(args.model, args.new_tokens, args.bias_phrases, args.boost)

    if rank == 0:
        out = {
            "metric": "audio-seconds/sec (RTF) + biased-WER, whisper-small 30s clips, batch32",
            "value": round(value, 2), "unit": "audio-seconds/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (seeded 30 s/16 kHz clips, random-init weights of the named architecture)",
            "config": {"workload": (f"{_config_tag(args, world)}: whisper-{args.model}, {B} clips/GPU x 30 s, log-mel + "
                                    f"encoder + {args.new_tokens}-token "
                                    f"{'greedy' if args.num_beams == 1 else f'beam-{args.num_beams}'} decode, "
                                    f"{args.bias_phrases}-phrase bias boost lambda={args.boost}")
                                   if not args.reference_mode else
                                   (f"reference mode: whisper-{args.model}, {B} clips/GPU x 30 s, log-mel + encoder + "
                                    f"greedy decode to natural EOS, max_length=225, no boost "
                                    f"(scripts/evaluation.py:173-179); batches serialised"),
                       "num_beams": args.num_beams, "global_batch": world * B, "parallelism": f"utterance-dp{world}",
                       "collective_backend": args.backend if world > 1 else None, "devices_used": devices_used,
                       "hipgraph_decode": use_graph, "batches_in_flight": 3 if overlap else 1},
            "rtf": round(1.0 / (value / world), 6),
            "roofline": roof if roof is not None else {"step": step_roof},
            "roofline_other": others or None,
            "phases": phases,
            # µs per launch of the lean decode projections inside the replayed decode graph (device stamps,
            # pipelined as the timed region), beside the serialised pass's phases above
            "decode_graph_launch_us": graph_us or None,
            "cpu_baseline": cpu,
            "biased_wer": bias_plumb,
        }
        if cpu:
            out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        if args.reference_mode:
            out["reference_mode"] = {"generated_tokens_per_clip": round(gen_tokens / (args.steps * B), 2),
                                     "ms_per_generated_token": round(ms_per_step / max(gen_tokens / args.steps / B, 1e-9), 4)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
