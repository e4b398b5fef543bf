#!/usr/bin/env python3
"""Benchmark of the Whisper contextual-biasing hot path on MI355X (BASELINE.json metric).

One "step" = the full inference path for one batch of synthetic 30 s / 16 kHz clips already
resident in HBM: log-mel → encoder → greedy decode of exactly 64 new tokens (EOS masked,
SURVEY.md §8(d) benchmark mode) with the fused bias-list boost (1000 phrases, lambda 2.0).
Default workload = config C2: whisper-small, batch 32 per GPU, bf16 (random-init weights of that
architecture; no checkpoint offline).

Multi-GPU (`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`): one process
per GPU, utterances sharded (weak scaling: 32 clips per GPU), weights generated on rank 0 and
broadcast once over RCCL/xGMI (`dist.broadcast`), no collective in the timed region besides the
barriers; time = max over ranks.

Prints ONE JSON line (rank 0) with the driver's contract fields plus `roofline` (dominant kernel:
the encoder MFMA GEMMs, timed with HIP events on the library's stream inside the timed region)
and `cpu_baseline` (the fp32 PyTorch-CPU restatement, both reference decode modes, timed on this
host, rank 0 / N=1 only).
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


def cpu_baseline(size: str, n_tokens: int, n_phr: int, boost: float, seed: int = 0, clips: int = 1):
    """the fp32 PyTorch-CPU restatement of the reference path (oracle/whisper_torch.py,
    test infrastructure) on the host cores, on a bounded sample of the same workload (log-mel + encoder
    + n_tokens greedy tokens with the same bias list and boost), in the reference's two decode modes:
    (i) use_cache=False exactly as scripts/evaluation.py:178 configures generate(), (ii) KV-cached.
    `value` is the faster mode (ii). One untimed warm-up clip, then `clips` timed clips per mode."""
    import torch
    from oracle import whisper_torch as WT
    from whisper_context_biasing_amd.config import get_dims
    from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list
    from whisper_context_biasing_amd.weights import make_weights
    dims = get_dims(size)
    m = WT.TorchWhisper(dims, make_weights(dims, seed=seed))
    pcm = torch.from_numpy(synth_batch(clips))
    phrases = synth_bias_list(n_phr, eot=dims.eos_token_id)
    kw = dict(max_length=n_tokens, min_new_tokens=n_tokens, bias=phrases, bias_boost=boost)

    def run(use_cache, n):
        t0 = time.perf_counter()
        mel = WT.log_mel(pcm[:n], dims.n_mel)
        m.generate(mel, use_cache=use_cache, **kw)
        return time.perf_counter() - t0

    with torch.no_grad():
        run(True, 1)                                  # warm-up (thread pool, allocator)
        t_cached = run(True, clips)
        t_nocache = run(False, clips)
    return {"value": round(clips * 30.0 / t_cached, 3), "unit": "audio-seconds/sec",
            "cores": torch.get_num_threads(), "kind": "port",
            "host_cpu_count": os.cpu_count(), "cpu_model": _cpu_model(),
            "modes": {"kv_cached": round(clips * 30.0 / t_cached, 3),
                      "use_cache_false_reference_config": round(clips * 30.0 / t_nocache, 3)},
            "sample": f"{clips} clip(s) x 30 s, whisper-{size} fp32 PyTorch-CPU restatement of the reference path "
                      f"(oracle/whisper_torch.py): log-mel + encoder + {n_tokens} greedy tokens with the "
                      f"{n_phr}-phrase boost; kv-cached {t_cached:.2f} s, use_cache=False "
                      f"(scripts/evaluation.py:178) {t_nocache:.2f} s wall; torch threads = the box's CPU share "
                      f"(OMP_NUM_THREADS), host has {os.cpu_count()} logical CPUs"}


def _pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass (profiles/*pmc*.json,
    written by tools/pmc_traffic.py: FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if kernel in d.get("kernels", {}):
            return d["kernels"][kernel]["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None


def _config_tag(args, world):
    """BASELINE.json configs: C2 small/32/greedy, C3 medium/64/beam-5, C4 small sharded, C5 large-v3/16/beam-5."""
    if args.num_beams > 1:
        return {"medium": "C3", "large-v3": "C5"}.get(args.model, "beam")
    return ("C4" if world > 1 else "C2") if args.model == "small" else "greedy"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
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
    ap.add_argument("--no-overlap", action="store_true",
                    help="serialise batches (default: batch i+1's front end + encoder overlap batch i's decode)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from whisper_context_biasing_amd.config import get_dims
    from whisper_context_biasing_amd.model import WhisperCB
    from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list
    from whisper_context_biasing_amd.shard import broadcast_weights, max_over_ranks, shard_bounds

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    dims = get_dims(args.model)
    # ---- weights: rank 0 generates, one RCCL broadcast of the packed bf16 blob over xGMI
    t0 = time.perf_counter()
    sd = broadcast_weights(dims, dev, seed=0)
    if world > 1:
        torch.cuda.synchronize()
        log(f"rank {rank}: weights broadcast in {time.perf_counter() - t0:.3f} s")
    model = WhisperCB.from_state_dict(dims, sd, dtype=args.dtype, device=local)
    del sd

    B = args.batch
    lo, hi = shard_bounds(world * B, rank, world)                      # this rank's utterances
    pcm = torch.from_numpy(synth_batch(hi - lo, start=lo)).to(dev)     # resident in HBM before timing
    phrases = synth_bias_list(args.bias_phrases, eot=dims.eos_token_id)
    bias = model.bias_list(phrases)
    use_graph = not args.no_graph

    overlap = not args.no_overlap
    keep = []   # async mode: inputs/outputs stay alive until the final synchronize

    def step():
        mel = model.log_mel(pcm)
        ids = model.generate(mel, max_length=args.new_tokens, min_new_tokens=args.new_tokens,
                             bias_list=phrases, bias_boost=args.boost, use_graph=use_graph, block=not overlap,
                             num_beams=args.num_beams)
        keep.append((mel, ids))
        return ids

    for i in range(args.warmup):
        ids = step()
        model.synchronize()
        torch.cuda.synchronize()
        log(f"warmup {i} done, ids {tuple(ids.shape)}")
    assert ids.shape[0] == B and (args.num_beams > 1 or ids.shape == (B, args.new_tokens))
    keep.clear()
    if not args.no_profile:
        # inside the timed region only the device stamps of the decode cross-attention are on (they
        # live in the kernel; HIP timing events on the library streams perturb the stream overlap)
        model.profile_enable(True, events=False, stamps=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    model.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * 30.0 / (elapsed / args.steps)
    prof, prof_steps = {}, args.steps
    if not args.no_profile:
        prof = model.profile_read()
        # phase breakdown + encoder GEMM timing: a separate, untimed pass with HIP events on every
        # front-end / encoder launch
        prof_steps = max(2, min(args.steps, 5))
        model.profile_enable(True, events=True, stamps=False)
        for i in range(prof_steps):
            step()
        model.synchronize()
        torch.cuda.synchronize()
        pass_prof = model.profile_read()
        model.profile_enable(False)
        keep.clear()
        pass_prof.pop("dec_xattn", None)
        for k, v in pass_prof.items():
            prof.setdefault(k, v)
    roofs = {}
    if prof.get("enc_gemm"):
        # encoder tile GEMMs: HIP events on the encoder stream around every launch
        p = prof["enc_gemm"]
        avg_ms = p["ms"] / p["launches"]
        achieved = p["flops"] / p["launches"] / (avg_ms * 1e-3) / 1e12
        peak = {"bf16": PEAK_BF16_TFLOPS, "f16": PEAK_F16_TFLOPS}.get(args.dtype, PEAK_F32_TFLOPS)
        kn = ("gemm_ring_kernel (encoder QKV/out/fc1/fc2/conv2, LDS-DMA ring; conv1 gemm_tile_kernel)"
              if args.dtype in ("bf16", "f16") else "gemm_tile_kernel (encoder conv/QKV/out/fc1/fc2)")
        roofs["enc_gemm"] = {"bound": "mfma", "kernel": kn,
                             "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                             "frac": round(achieved / peak, 4), "traffic": None,
                             "avg_launch_ms": round(avg_ms, 4), "flops_per_launch": p["flops"] / p["launches"],
                             "total_ms_per_step": round(p["ms"] / prof_steps, 3),
                             "timing": "hip_events (separate profiled pass of the same step)"}
    if prof.get("dec_xattn"):
        # decode cross-attention: replayed inside the decode hipGraph, so each launch is timed by
        # s_memrealtime stamps (first workgroup start → last workgroup end) written by the kernel
        p = prof["dec_xattn"]
        avg_ms = p["ms"] / p["launches"]
        bpl = p["bytes"] / p["launches"]
        achieved = bpl / (avg_ms * 1e-3) / 1e9
        xenc = args.dtype in ("bf16", "f16") and dims.d_model <= 1024 and os.environ.get("WCB_XMODE", "1") != "0" \
            and (args.num_beams == 1 or os.environ.get("WCB_BEAM_XMODE", "0") == "1")
        kname = ("attn_xenc_kernel (decoder cross-attention in encoder space: one pass over the encoder "
                 "output per layer for all heads)") if xenc else \
            "attn_decode2p_kernel / attn_decode_kernel (decoder cross-attention over precomputed per-layer K/V; " \
            "single-pass kernel when a launch has <= 2048 (row, head) workgroups)"
        roofs["dec_xattn"] = {"bound": "hbm", "kernel": kname,
                              "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                              "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                              "avg_launch_ms": round(avg_ms, 4), "bytes_per_launch": bpl,
                              "total_ms_per_step": round(p["ms"] / args.steps, 3),
                              "timing": "device s_memrealtime stamps (graph node), inside the timed region"}
    roof = None
    if roofs:
        dom = max(roofs, key=lambda k: roofs[k]["total_ms_per_step"])   # dominant = most kernel time
        roof = dict(roofs[dom])
        # the committed PMC pass (tools/measure.sh) measures the default C2 workload only
        c2 = (args.model, args.batch, args.num_beams, args.dtype, args.new_tokens) == ("small", 32, 1, "bf16", 64)
        tr = _pmc_traffic(dom) if c2 else None
        if tr:
            roof["traffic"], roof["traffic_source"] = tr
        others = {k: v for k, v in roofs.items() if k != dom}
    phases = {k: {"ms_per_step": round(v["ms"] / (args.steps if k == "dec_xattn" else prof_steps), 3),
                  "launches_per_step": v["launches"] / (args.steps if k == "dec_xattn" else prof_steps)}
              for k, v in prof.items()}

    # biased-WER half of the metric, as a plumbing check (random weights: no transcript to score
    # against): the boosted decode of the last batch against a λ = 0 decode of the same clips, scored
    # by the C++ host scorer with token ids as words (WER, and compute_bias_wer's tallies over the
    # bias phrases), untimed
    bias_plumb = None
    if rank == 0 and args.boost > 0:
        from whisper_context_biasing_amd.metrics import wer_counts
        import ctypes as C
        from whisper_context_biasing_amd import _lib
        from whisper_context_biasing_amd.metrics import _cstrs
        mel = model.log_mel(pcm)
        kw = dict(max_length=args.new_tokens, min_new_tokens=args.new_tokens, use_graph=use_graph,
                  num_beams=args.num_beams)
        boosted = model.generate(mel, bias_list=phrases, bias_boost=args.boost, **kw).cpu().tolist()
        plain = model.generate(mel, **kw).cpu().tolist()
        model.synchronize()
        as_text = lambda rows: [" ".join(map(str, r)) for r in rows]
        err, words = wer_counts(as_text(boosted), as_text(plain))
        ptxt = [" ".join(map(str, p)) for p in phrases]
        bd = bt = 0
        for r, h in zip(as_text(boosted), as_text(plain)):   # phrases the boost placed, lost without it
            d_, t_ = C.c_int64(), C.c_int64()
            _lib.check(_lib.load().wcb_bias_counts((" " + r + " ").encode(), (" " + h + " ").encode(),
                                                   _cstrs([" " + t + " " for t in ptxt]), len(ptxt),
                                                   C.byref(d_), C.byref(t_)), None, "wcb_bias_counts")
            bd += d_.value
            bt += t_.value
        bias_plumb = {"wer_boosted_vs_unboosted": round(100.0 * sum(err) / max(sum(words), 1), 3),
                      "bias_wer_unboosted_vs_boosted": round(100.0 * bd / bt, 3) if bt else 0.0,
                      "bias_phrase_tokens_in_boosted": bt,
                      "note": "plumbing only (random weights): token ids as words; WER of the boosted decode "
                              "against the λ=0 decode, bias-WER of the λ=0 decode against the boosted one"}

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
            "config": {"workload": f"{_config_tag(args, world)}: whisper-{args.model}, {B} clips/GPU x 30 s, log-mel + "
                                   f"encoder + {args.new_tokens}-token "
                                   f"{'greedy' if args.num_beams == 1 else f'beam-{args.num_beams}'} decode, "
                                   f"{args.bias_phrases}-phrase bias boost lambda={args.boost}",
                       "num_beams": args.num_beams, "global_batch": world * B, "parallelism": f"utterance-dp{world}",
                       "hipgraph_decode": use_graph, "batches_in_flight": (int(os.environ.get("WCB_DECODE_CTX", "2")) + 1) if overlap else 1},
            "rtf": round(1.0 / (value / world), 6),
            "roofline": roof,
            "roofline_other": others if roofs else None,
            "phases": phases,
            "cpu_baseline": cpu,
            "biased_wer": bias_plumb,
        }
        if cpu:
            out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
