#!/usr/bin/env python
"""Headline benchmark: SimCSE/DuoRec contrastive train step of the user tower at the batch
BASELINE.json's metric names ("SimCSE train-step pairs/sec at d=128, batch 8192"), 1 x MI355X.

A step = one full training step of tower_code/v1_usertower_train.py:717-893 on one global
batch of synthetic H&M-shaped users: two dropout views (p=0.2) of SASRecUserTower, the
all-time-steps LogQ in-batch loss (N ~ 153k valid positions at 8192 users, N x N implicit
logits), DuoRec (InfoNCE + SupCon), backward, clip_grad_norm_(5.0), AdamW (item matrix
unfrozen, lr x 0.05: the reference's epoch >= 2 steady state). Inputs are resident in HBM
before timing. Secondary lines: batch 4096 (configs[1]), the fp32 parity mode, batch 32768 on
one GPU, DeepFM (configs[2]), retrieve->rerank (configs[4] on one GPU), the item tower
(configs[0] shape), HNM; the CPU oracle on the headline's own batch (cpu_baseline).

Multi-GPU (one process per GPU, RCCL): ``--gpus N`` without torchrun's environment starts
``torch.distributed.run --nproc-per-node N`` as a child process (this parent never touches
the GPU); under torchrun each rank holds 8192 users by default, so the global batch is
8192 x N (weak scaling; N=4 is configs[3]'s global batch 32768, negatives all-gathered).
``--batch G`` fixes the global batch instead (strong scaling). Users are split by rank; see
dist.py. At every N the JSON also carries ``strong_32768`` (configs[3]: the FIXED global batch
32768 split over the N ranks; at N > 1 with rank 0's one-GPU run of the same batch in the same
process and the speedup over it) and, at N > 1, ``retrieve_rerank_sharded`` (configs[4]: the 1M
corpus sharded by item range, merged top-100 over RCCL, DeepFM rerank sharded by query).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32-input MFMA (= f32 vector peak)
BF16_MFMA_PEAK_TFLOPS = 16 * FP32_MFMA_PEAK_TFLOPS  # 2516.8: dense bf16 MFMA (16x the f32 rate, same guide)
# bf16x3: every fp32-equivalent FLOP is three bf16 MFMA products (hi*hi + hi*lo + lo*hi)
BF16X3_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 3
# f16 loss mode: logits 3 fp16 MFMAs per product, gradient products 1: 2 MFMA passes per algorithmic FLOP
F16_SPLIT_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 2
TRAFFIC_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06_nce_fwdg_h_traffic_b8192.json")
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU, RCCL). Without torchrun's env this process starts "
                         "`torch.distributed.run --nproc-per-node N` as a child and exits with its code")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="fixed global batch (users) for every N: strong scaling. Default: --batch-per-gpu x N")
    ap.add_argument("--batch-per-gpu", type=int, default=8192,
                    help="users per GPU when --batch is not given (weak scaling). N=1: the 8192-user batch "
                         "BASELINE.json's metric names; N=4: configs[3]'s global batch 32768")
    ap.add_argument("--items", type=int, default=47_062)
    ap.add_argument("--dropout", type=float, default=0.2)
    ap.add_argument("--freeze-items", action="store_true", help="epoch-1 regime (item matrix frozen)")
    ap.add_argument("--cpu-loss-chunk", type=int, default=64,
                    help="row chunk of the CPU oracle's N x N main loss (same arithmetic, bounded RAM)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads; 0 = the host's physical cores (BASELINE.md), capped by the CPUs "
                         "this process may use (affinity mask and cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-batch4096", action="store_true",
                    help="skip the secondary line at global batch 4096 (BASELINE configs[1])")
    ap.add_argument("--steps4096", type=int, default=10)
    ap.add_argument("--no-batch32768", action="store_true",
                    help="skip the N=1 run of configs[3]'s global batch 32768 (the strong-scaling baseline)")
    ap.add_argument("--steps32768", type=int, default=3)
    ap.add_argument("--no-fp32-line", action="store_true",
                    help="skip the secondary line in the fp32 parity mode (fp32 MFMA loss, fp32 GEMMs/attention)")
    ap.add_argument("--steps-fp32", type=int, default=3)
    ap.add_argument("--no-deepfm", action="store_true", help="skip the DeepFM rerank secondary metric")
    ap.add_argument("--deepfm-rows", type=int, default=65536)
    ap.add_argument("--deepfm-vocab", type=int, default=1_000_000)
    ap.add_argument("--no-rerank", action="store_true", help="skip the retrieve->rerank secondary metric")
    ap.add_argument("--corpus", type=int, default=1_000_000, help="retrieve->rerank corpus size")
    ap.add_argument("--no-item-tower", action="store_true", help="skip the item-tower secondary metric")
    ap.add_argument("--nce-precision", default="f16", choices=["f16", "bf16x3", "fp32"],
                    help="precision of the grouped LogQ loss kernels (ops.set_nce_precision): f16 = fp16x3 logits "
                         "and single-fp16-MFMA gradient products (default), bf16x3 = both products as three bf16 "
                         "MFMAs, fp32 = fp32-input MFMA")
    ap.add_argument("--no-prefetch-index", action="store_true",
                    help="build each batch's index inside its own step (host syncs mid-step)")
    ap.add_argument("--unfused-adamw", action="store_true", help="torch's foreach AdamW instead of fused")
    ap.add_argument("--blas", default="default", choices=["default", "hipblaslt", "rocblas", "ck"],
                    help="library torch uses for the tower's dense projections")
    ap.add_argument("--master-port", type=int, default=29531, help="rendezvous port when spawning ranks")
    ap.add_argument("--rehearse-one-device", action="store_true",
                    help="rehearsal of the N>1 code path on a 1-GPU box: every rank on cuda:0, gloo transport "
                         "(numbers are not scaling results)")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """--gpus N > 1 without torchrun's environment: start torchrun as a CHILD process (one rank per
    GPU, rendezvous on 127.0.0.1) and return its exit code. This parent never touches the GPU."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={args.master_port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    if world > 1 and args.rehearse_one_device:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group(backend="gloo", init_method="env://", rank=rank, world_size=world)
        return rank, world, torch.device("cuda", 0)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", init_method="env://", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
    else:
        torch.cuda.set_device(0)
    return rank, world, torch.device("cuda", local if world > 1 else 0)


def host_cpu_info():
    """os.cpu_count(), the lscpu model name and the physical core count of this host."""
    info = {"os_cpu_count": os.cpu_count(), "model": None, "physical_cores": None}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {}
        for line in out.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                kv[k.strip()] = v.strip()
        info["model"] = kv.get("Model name")
        cps, sock = kv.get("Core(s) per socket"), kv.get("Socket(s)")
        if cps and sock and cps.isdigit() and sock.isdigit():
            info["physical_cores"] = int(cps) * int(sock)
    except (OSError, ValueError):
        pass
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:  # cgroup v2 CPU bandwidth quota ("max 100000" = unlimited)
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            info["cgroup_cpu_quota"] = round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        pass
    return info


class _Heartbeat:
    """Prints a progress line to stderr every `every` seconds while a long host-only phase runs
    (the GPU box takes a command that is silent for minutes to be hung)."""

    def __init__(self, what, every=20.0):
        import threading
        self.what, self.every, self.t0 = what, every, time.perf_counter()
        self.stop = threading.Event()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(self.every):
            print(f"[bench] {self.what}: {time.perf_counter() - self.t0:.0f} s", file=sys.stderr, flush=True)

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()
        return False


def _walk_clocks(obj, out, path=""):
    """Collect {path: MHz} for every clock entry of an amd-smi / rocm-smi JSON document."""
    if isinstance(obj, dict):
        for k, v in obj.items():
            _walk_clocks(v, out, f"{path}/{k}")
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            _walk_clocks(v, out, f"{path}[{i}]")
    else:
        import re
        low = path.lower()
        if ("clk" in low or "clock" in low) and not any(w in low for w in ("min_", "max_", "_locked", "deep_sleep",
                                                                          "level")):
            m = re.search(r"([0-9]+(?:\.[0-9]+)?)", str(obj))
            if m and (low.endswith("/value") or "mhz" in str(obj).lower() or low.endswith("clock speed:")):
                out[path] = float(m.group(1))


def gpu_clocks():
    """Shader (SCLK) and memory (MCLK) clocks of the visible GPU right now, from amd-smi (rocm-smi as a
    fallback): {"sclk_mhz", "mclk_mhz", "source"} (None where the tool or field is missing). Bench lines
    from different boxes are only comparable at equal clocks."""
    import subprocess
    res = {"sclk_mhz": None, "mclk_mhz": None, "source": None}
    for cmd in (["amd-smi", "metric", "-c", "--json"], ["rocm-smi", "--showclocks", "--json"]):
        try:
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=20)
            out = p.stdout
            start = min([i for i in (out.find("{"), out.find("[")) if i >= 0], default=-1)
            if start < 0:
                continue
            doc = json.JSONDecoder().raw_decode(out[start:])[0]  # the tools may print warnings around it
        except (OSError, ValueError, subprocess.SubprocessError):
            continue
        flat = {}
        _walk_clocks(doc, flat)
        sc = [v for k, v in flat.items() if any(w in k.lower() for w in ("gfx", "sclk"))]
        mc = [v for k, v in flat.items() if any(w in k.lower() for w in ("/mem", "mclk"))]
        if sc or mc:
            # amd-smi reports one shader clock per XCD (gfx_0..gfx_7): their mean, and the spread
            res.update({"sclk_mhz": round(sum(sc) / len(sc), 1) if sc else None,
                        "sclk_range_mhz": [min(sc), max(sc)] if sc else None,
                        "mclk_mhz": max(mc) if mc else None, "source": " ".join(cmd[:2])})
            break
    return res


def cpu_threads(args):
    """(threads, host info, rule): BASELINE.md's P = physical host cores, capped by this
    process's affinity mask and cgroup CPU quota (the GPU box grants a share of the host)."""
    info = host_cpu_info()
    phys = info.get("physical_cores") or os.cpu_count() or 1
    avail = min(info.get("affinity_cpus") or phys, int(info.get("cgroup_cpu_quota") or phys))
    threads = max(1, min(args.cpu_threads or phys, phys, avail))
    rule = ("physical cores (BASELINE.md), capped by this process's affinity mask / cgroup CPU quota: "
            f"physical {phys}, usable {avail}")
    return threads, info, rule


def cpu_timed(fn, warm=2, reps=5, single_over_s=60.0):
    """BASELINE.md's CPU timing rule: `warm` untimed calls, then the median of `reps` timed calls
    (one timed call when a call takes longer than single_over_s). -> (median s, timed calls)."""
    t0 = time.perf_counter()
    fn()
    first = time.perf_counter() - t0
    if first > single_over_s:
        return first, 1
    for _ in range(warm - 1):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], reps


def gpu_step_from_state(state, cfg, items, batch, device):
    """One GPU train step exactly as the headline times it (dist.contrastive_step_dp: packed two-view
    tower, grouped LogQ + DuoRec kernels, backward, native clip + AdamW) from a given state -- the
    oracle's tower weights, item matrix and AdamW moments (state["model"], ["W"], ["opt"]) -- at dropout
    0 on `batch` (CPU tensors). -> oracle.agreement.capture of the result (CPU copies)."""
    import dataclasses
    from oracle import agreement as OA
    from recsys_amd import dist as D
    from recsys_amd.tower_code import v1_usertower_train as TT
    from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
    cfg0 = dataclasses.replace(cfg, dropout=0.0)
    model = SASRecUserTower(cfg0).to(device)
    model.load_state_dict(state["model"])
    model.train()
    W = state["W"]
    it = TT.SASRecItemTower(W.shape[0] - 1, W.shape[1], items.log_q.clone()).to(device)
    it.init_from_pretrained(W.to(device))
    it.set_freeze_state(False)
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay, fused=True)
    opt.add_param_group({"params": list(it.parameters()), "lr": cfg.lr * 0.05})
    opt.load_state_dict(state["opt"])
    bucket = D.GradBucket(list(model.parameters()) + list(it.parameters()))
    bd = {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in batch.items()}
    lookup = items.pretrained.to(device)
    ix = D.prepare_step_index(bd, pretrained_lookup=lookup)
    losses = D.contrastive_step_dp(model, it, it.log_q, bd, opt, cfg0, lookup, bucket, index=ix)
    torch.cuda.synchronize()
    return OA.capture(model, it.item_matrix.weight, losses)


def oracle_state(model, W, opt):
    """CPU copies of the oracle's step state (what gpu_step_from_state starts from)."""
    import copy
    return {"model": {k: v.detach().clone() for k, v in model.state_dict().items()}, "W": W.detach().clone(),
            "opt": copy.deepcopy(opt.state_dict())}


def cpu_baseline(args, items, cfg, batch_size, batch_seed, device=None):
    """The oracle (CPU PyTorch fp32 restatement of tower_code/v1_usertower_train.py:717-893) on
    the SAME global batch the GPU headline runs (same generator, same seed), dropout p = 0
    (BASELINE.md): one timed step after a small warm-up step; the main loss row-chunked (same
    arithmetic, bounded RAM). With `device`, the GPU step is then run from the oracle's own pre-step
    state (weights, item matrix, AdamW moments after the warm-up) on the same batch at dropout 0, and
    the two results are compared (oracle/agreement.py: losses 1e-4, gradients 1e-3 of scale,
    post-AdamW parameters 1e-5): "agreement_with_gpu"."""
    import dataclasses
    from oracle import agreement as OA
    from oracle import user_tower as O
    from recsys_amd import synth
    threads, info, rule = cpu_threads(args)
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(args.seed)
    cfg = dataclasses.replace(cfg, dropout=0.0)
    model = O.OracleUserTower(cfg)
    model.train()
    W = torch.nn.Parameter(items.pretrained.clone())
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay)
    opt.add_param_group({"params": [W], "lr": cfg.lr * 0.05})
    warm = synth.make_batch(items, 64, seed=args.seed + 7)
    O.contrastive_step(model, W, items.log_q, warm, opt, items.pretrained, loss_chunk=args.cpu_loss_chunk)
    batch = synth.make_batch(items, batch_size, seed=batch_seed)
    n_valid = int((~batch["padding_mask"]).sum())
    state = oracle_state(model, W, opt) if device is not None else None
    with _Heartbeat(f"cpu_baseline step ({batch_size} users, {n_valid} valid steps)"):
        t0 = time.perf_counter()
        losses = O.contrastive_step(model, W, items.log_q, batch, opt, items.pretrained,
                                    loss_chunk=args.cpu_loss_chunk)
        dt = time.perf_counter() - t0
    torch.set_num_threads(prev_threads)
    out = {"value": round(batch_size / dt, 3), "unit": "pairs/s", "cores": threads,
           "kind": "port",
           "threads_rule": rule,
           "host": info,
           "sample": (f"oracle/user_tower.py contrastive_step (fp32 PyTorch CPU, dropout 0, AdamW) on the GPU "
                      f"headline's first global batch ({batch_size} users, {n_valid} valid steps, same seed); "
                      f"ONE timed step ({dt:.1f} s) after a 64-user warm-up step; main loss evaluated over "
                      f"{args.cpu_loss_chunk}-row chunks of the N x N logits under activation checkpointing "
                      f"(same per-element arithmetic; the one-shot N x N tensors would need ~{4 * n_valid ** 2 / 1e9:.0f} GB)"),
           "seconds_per_step": round(dt, 2)}
    if device is not None:
        ref = OA.capture(model, W, losses)
        dut = gpu_step_from_state(state, cfg, items, batch, device)
        agr = OA.compare_step(ref, dut)
        agr["what"] = ("the GPU step (dist.contrastive_step_dp, dropout 0) from the oracle's pre-step state on the "
                       "same batch vs this timed oracle step: losses, clipped gradients, post-AdamW parameters")
        out["agreement_with_gpu"] = agr
        assert agr["ok"], agr
    return out


def deepfm_cpu_state(model):
    """Host copies of a DeepFM module's tables and DNN weights (the CPU baselines' inputs)."""
    names = model.field_names
    with torch.no_grad():
        return {"emb": [model.embedding_dict[n].weight.detach().cpu() for n in names],
                "lin": [model.linear_model.embedding_dict[n].weight.detach().cpu() for n in names],
                "ws": [m.weight.detach().cpu() for m in model.dnn.linears],
                "bs": [m.bias.detach().cpu() for m in model.dnn.linears],
                "wo": model.dnn_linear.weight.detach().cpu(), "bias": float(model.out.bias.item())}


def _deepfm_cpu(st, x):
    from oracle import deepfm as OD
    return OD.deepfm_forward(x, st["emb"], st["lin"], st["bias"], st["ws"], st["bs"], st["wo"], dtype=torch.float32)


def cpu_baseline_deepfm(args, st, x, gpu_logits=None):
    """configs[2] on the host: oracle/deepfm.py (gather + FM + DNN, fp32) on the GPU line's own
    65,536 Zipf(1.1) rows over the same 39 x 1e6-row tables. With gpu_logits (the GPU line's output
    for the same rows), the timed call's logits are compared with it: "agreement_with_gpu" (every
    row within 1e-4, the north star's logit tolerance; asserted)."""
    threads, info, rule = cpu_threads(args)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    xc = x.cpu()
    res = {}

    def call():
        res["out"] = _deepfm_cpu(st, xc)

    with torch.no_grad(), _Heartbeat("cpu_baseline deepfm"):
        dt, n = cpu_timed(call)
    torch.set_num_threads(prev)
    R = xc.shape[0]
    out = {"value": round(R / dt, 1), "unit": "rows/s", "cores": threads, "kind": "port", "threads_rule": rule,
           "sample": (f"oracle/deepfm.py deepfm_forward (fp32 PyTorch CPU: 39 table gathers, FM, DNN 624-256-128-1) "
                      f"on the GPU line's {R} rows (the whole batch, same ids and tables); median of {n} calls "
                      f"after 2 warm-up calls"),
           "seconds_per_call": round(dt, 4)}
    if gpu_logits is not None:
        ref = res["out"][0].reshape(-1).double()
        got = gpu_logits.detach().reshape(-1).double().cpu()
        err = (got - ref).abs()
        out["agreement_with_gpu"] = {"rows": R, "logit_max_abs_err": float(err.max()),
                                     "logit_mean_abs_err": float(err.mean()), "tol": 1e-4,
                                     "ok": bool(float(err.max()) <= 1e-4)}
        assert out["agreement_with_gpu"]["ok"], out["agreement_with_gpu"]
    return out


def cpu_baseline_retrieve_rerank(args, st, gpu_out, Qs=512, K=100, F=39, chunk=250_000):
    """configs[4] on the host, one rank's worth (the whole 1M corpus): oracle/ranker.py
    retrieve_rerank -- the reference arithmetic scores = user @ items.T in fp32 + torch.topk(100)
    (v1_usertower_train.py:672-675, ranker_skelet.py:193-196; items in 250k-row chunks, per-chunk
    top-100 merged) + the same hashed rerank ids + oracle DeepFM + top-10 -- for the first Qs of the
    GPU line's 4,096 queries (same seed-5 corpus and users). queries/s. The timed call's output is
    then checked against the GPU line's own output for those queries (oracle.ranker.compare_rerank:
    candidate sets, final ids up to ranker near-ties, final scores within 1e-5)."""
    from oracle import ranker as ORK
    threads, info, rule = cpu_threads(args)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    I, V = args.corpus, args.deepfm_vocab
    g = torch.Generator(device="cpu").manual_seed(5)
    corpus = torch.nn.functional.normalize(torch.randn(I, 128, generator=g), dim=1)
    users = torch.nn.functional.normalize(torch.randn(4096, 128, generator=g), dim=1)[:Qs].contiguous()
    bucket = torch.arange(Qs, dtype=torch.int64) % 1000
    res = {}

    def step():
        res["out"] = ORK.retrieve_rerank(users, corpus, st, [V] * F, k=K, final_k=10, user_bucket=bucket,
                                         chunk=chunk)

    with torch.no_grad(), _Heartbeat("cpu_baseline retrieve->rerank"):
        dt, n = cpu_timed(step)
    torch.set_num_threads(prev)
    _, ci, p_all, top_ref, _ = res["out"]
    ids, p, cand = (t[:Qs].cpu() for t in gpu_out)
    check = ORK.compare_rerank(ids, p, cand, ci, top_ref, p_all, p_tol=1e-5)
    assert check["same_candidate_set"] >= int(0.95 * Qs), check
    return {"value": round(Qs / dt, 1), "unit": "queries/s", "cores": threads, "kind": "port", "threads_rule": rule,
            "sample": (f"oracle/ranker.py retrieve_rerank: fp32 matmul + torch.topk({K}) over the {I}-item corpus "
                       f"({chunk}-item chunks, merged) + hashed rerank ids + oracle/deepfm.py on {Qs}x{K} rows + "
                       f"top-10, for the first {Qs} of the GPU line's 4,096 queries (same corpus and users); median "
                       f"of {n} calls after 2 warm-up calls"),
            "seconds_per_call": round(dt, 4),
            "agreement_with_gpu": check}


def cpu_baseline_item_tower(args, gpu_model, inputs):
    """configs[0] as BASELINE.md specifies it (its own CPU-runnable case): oracle/item_tower.py
    OracleHybridItemTower forward (eval) on 256 items, d = 64, with the GPU line's weights (the
    bert-base-shaped local BERT included) and inputs. items/s."""
    import copy
    from oracle import item_tower as OIT
    threads, info, rule = cpu_threads(args)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    bert = copy.deepcopy(gpu_model.bert_model).cpu()
    ref = OIT.OracleHybridItemTower(gpu_model.std_embedding.num_embeddings, gpu_model.std_field_emb.shape[1],
                                    gpu_model.embed_dim, gpu_model.head.final_proj.out_features, bert_model=bert)
    ref.load_state_dict({k: v.detach().cpu() for k, v in gpu_model.state_dict().items()})
    ref.eval()
    xs = [t.cpu() for t in inputs]
    res = {}

    def call():
        res["out"] = ref(*xs)

    with torch.no_grad(), _Heartbeat("cpu_baseline item tower"):
        dt, n = cpu_timed(call, warm=1, reps=3)
    torch.set_num_threads(prev)
    B = xs[0].shape[0]
    out = {"value": round(B / dt, 1), "unit": "items/s", "cores": threads, "kind": "port", "threads_rule": rule,
           "sample": (f"oracle/item_tower.py OracleHybridItemTower forward (fp32 PyTorch CPU, eval) on the GPU "
                      f"line's {B} items and weights (bert-base-shaped local BERT, all 12 layers); median of {n} "
                      f"calls after 1 warm-up call"),
           "seconds_per_call": round(dt, 4)}
    # the timed call's output against the GPU module's on the same inputs (eval, same weights):
    # atol 1e-5 / rtol 1e-4 (tests/test_gpu_item_tower.py's bound, here through all 12 BERT layers)
    with torch.no_grad():
        got = gpu_model(*inputs).float().cpu()
    exp = res["out"].float()
    err = (got - exp).abs()
    bound = 1e-5 + 1e-4 * exp.abs()
    out["agreement_with_gpu"] = {"items": B, "max_abs_err": float(err.max()),
                                 "max_err_over_bound": float((err / bound).max()), "atol": 1e-5, "rtol": 1e-4,
                                 "ok": bool((err <= bound).all())}
    assert out["agreement_with_gpu"]["ok"], out["agreement_with_gpu"]
    return out


def bench_deepfm(args, device):
    """BASELINE configs[2]: DeepFM forward, 65,536 rows x 39 sparse fields, d=16, per-field
    vocab 1e6, Zipf(1.1) ids. rows/s with inputs resident in HBM."""
    import numpy as np
    from recsys_amd import ops
    from recsys_amd.temp_model.ranker_skelet import DeepFM
    R, F, V = args.deepfm_rows, 39, args.deepfm_vocab
    model = DeepFM([V] * F, device=device)
    rng = np.random.default_rng(args.seed + 3)
    x = torch.from_numpy(((rng.zipf(1.1, size=(R, F)) - 1) % V).astype(np.int64)).to(device)
    for _ in range(3):
        model.forward_logits(x)
    torch.cuda.synchronize()
    iters = 20
    ops.timing_start()
    t0 = time.perf_counter()
    for _ in range(iters):
        model.forward_logits(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    kt = ops.timing_stop()
    # the fused kernel (gather + FM + DNN in one launch): algorithmic HBM bytes per row =
    # SURVEY.md 8d's 39 x (64 B embedding row + 4 B first-order weight + 8 B id) + 4 B output =
    # 2,968 B; DNN FLOPs per row 2 (624*256 + 256*128 + 128), priced at the bf16x3 MFMA peak
    f_n, f_ms = kt.get("deepfm/fused", (0, 0.0))
    bytes_row = F * (64 + 4 + 8) + 4
    dnn_flops = 2.0 * R * (F * 16 * 256 + 256 * 128 + 128)
    out = {"metric": "DeepFM rerank rows/sec (forward, 39 fields, d=16, vocab 1e6/field)",
           "value": round(R / dt, 1), "unit": "rows/s", "rows": R, "ms_per_batch": round(dt * 1e3, 4),
           "data": "synthetic Zipf(1.1) ids, deepctr-style N(0,1e-4) init"}
    if f_n:
        fs = f_ms / 1e3 / f_n
        out["fused"] = {"kernel": "deepfm_rows2m_k<39, 1> (F = 39: eight 32-row waves per 256-row workgroup; deepfm_rows5_k on unpacked tables, deepfm_persist_k for other F in [25, 48], deepfm_fused_k otherwise) on cached packed tables and weight images", "avg_ms": round(fs * 1e3, 4),
                        "bytes_per_row": bytes_row,
                        "gather_achieved_GBs": round(bytes_row * R / fs / 1e9, 1), "hbm_peak_GBs": HBM_PEAK_GBS,
                        "gather_frac": round(bytes_row * R / fs / 1e9 / HBM_PEAK_GBS, 4),
                        "dnn_achieved_TFLOPs": round(dnn_flops / fs / 1e12, 2),
                        "dnn_peak_TFLOPs": round(BF16X3_PEAK_TFLOPS, 1),
                        "dnn_frac": round(dnn_flops / fs / 1e12 / BF16X3_PEAK_TFLOPS, 4)}
    else:
        emb_n, emb_ms = kt.get("deepfm/embed", (1, 0.0))
        lin_n, lin_ms = kt.get("deepfm/linear", (1, 0.0))
        dot_n, dot_ms = kt.get("deepfm/linear_dot", (1, 0.0))
        eb = F * 8 + F * 17 * 4 + F * 16 * 4 + 4   # + the 624-float DNN input row written
        emb_s = emb_ms / 1e3 / emb_n
        dnn_s = (lin_ms / lin_n + dot_ms / dot_n) / 1e3
        out["gather_fm"] = {"avg_ms": round(emb_s * 1e3, 4), "bytes_per_row": eb,
                            "achieved_GBs": round(eb * R / emb_s / 1e9, 1), "peak_GBs": HBM_PEAK_GBS,
                            "frac": round(eb * R / emb_s / 1e9 / HBM_PEAK_GBS, 4)}
        out["dnn"] = {"avg_ms": round(dnn_s * 1e3, 4), "achieved_TFLOPs": round(dnn_flops / dnn_s / 1e12, 2),
                      "peak_TFLOPs": FP32_MFMA_PEAK_TFLOPS,
                      "frac": round(dnn_flops / dnn_s / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)}
    # uniform-id stress variant: every row gathers cold table lines
    xu = torch.randint(0, V, (R, F), device=device, generator=torch.Generator(device=device).manual_seed(9))
    for _ in range(3):
        model.forward_logits(xu)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        model.forward_logits(xu)
    torch.cuda.synchronize()
    out["uniform_ids_rows_per_s"] = round(R / ((time.perf_counter() - t0) / iters), 1)
    return model, out, x


def bench_gather_1m(device, T=316_372, rows=1_000_000, iters=10, flush_mb=1024):
    """The embedding gather on DRAM-resident rows (SURVEY.md 7 "cache effects"): the fused
    seq-embed forward (seq_embed_fwd_k, the north star's ">= 40 % of HBM on embedding gather")
    over T packed tokens (the headline launch's size: both dropout views of the 8192-user batch)
    with a 1M-row item-id table (512 MB, past the 256 MB Infinity Cache) and uniform ids, a fresh
    projected-pretrained base per token, the reference's gates (s_mask: item-id and time tables
    live, side tables 0), position add, LayerNorm and dropout 0.2. A 1 GiB buffer is written
    before every launch so neither the table, the base nor the output stays cache-resident, and
    each launch is timed alone with HIP events on its stream. Algorithmic bytes per token: base
    row 512 + item row 512 + output row 512 + ids/position 24 + mean/rstd 8 = 1,568 B; the
    12-row time table is read too but credited with nothing (it is cache-resident by nature)."""
    from recsys_amd import ops
    D, L = 128, 50
    g = torch.Generator(device="cpu").manual_seed(21)
    base = torch.randn(T, D, generator=g).to(device)
    item_ids = torch.randint(1, rows, (T,), generator=g).to(device)
    time_ids = torch.randint(1, 10, (T,), generator=g).to(device)
    side = [torch.randint(1, 1001, (T,), generator=g).to(device) for _ in range(4)]
    tok_pos = torch.randint(0, L, (T,), generator=g).to(device)
    item_tab = (0.02 * torch.randn(rows, D, generator=g)).to(device)
    time_tab = (0.02 * torch.randn(12, D, generator=g)).to(device)
    side_tab = [(0.02 * torch.randn(1001, D, generator=g)).to(device) for _ in range(4)]
    gate = torch.tensor([0.5, 0.5, 0.0, 0.0, 0.0, 0.0], device=device)
    pos = (0.02 * torch.randn(L, D, generator=g)).to(device)
    ln_w, ln_b = torch.ones(D, device=device), torch.zeros(D, device=device)
    scratch = torch.empty(flush_mb << 18, device=device, dtype=torch.float32)
    ids = [item_ids, time_ids] + side
    tabs = [item_tab, time_tab] + side_tab
    ms = []
    with torch.no_grad():
        for i in range(iters + 2):
            scratch.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ops.seq_embed(base, ids, tabs, gate, pos, ln_w, ln_b, p_drop=0.2, padding_idx=[0] * 6, tok_pos=tok_pos)
            b.record()
            torch.cuda.synchronize()
            if i >= 2:
                ms.append(a.elapsed_time(b))
    avg = sum(ms) / len(ms)
    bpt = 512 * 3 + 24 + 8
    ach = bpt * T / (avg / 1e3) / 1e9
    return {"kernel": "seq_embed_fwd_k", "bound": "hbm", "tokens_per_launch": T, "table_rows": rows,
            "bytes_per_token": bpt, "avg_launch_ms": round(avg, 4), "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "note": "uniform ids over a 512 MB table, 1 GiB cache flush before each launch, time table uncredited"}


def bench_retrieve_rerank(args, device, deepfm, rank=0, world=1):
    """BASELINE configs[4]: Q=4096 normalised user vectors against a 1M-item normalised corpus
    (seed 5), ReRankingSystem.recommend_batch: top-100 by rsx_retrieve_topk, 39 hashed (user
    bucket, item) sparse ids per candidate (hashed_cross_features), DeepFM on the Q x 100 rows,
    final top-10 per query by probability. queries/s; the retrieval op priced at the dense bf16
    MFMA peak.

    world > 1: the corpus is sharded by item range (I/N rows per rank); every rank
    scores all Q queries against its shard, the [Q, 100] (score, global index) lists are
    all-gathered over RCCL and merged by (score desc, index asc) (dist.retrieve_topk_sharded);
    the DeepFM rerank is sharded by query (rank r reranks queries [r Q/N, (r+1) Q/N),
    ReRankingSystem.rerank_batch). The step time is the max over ranks; value = Q / that time.
    Returns (line, (final ids, final scores, candidates) of this rank's queries)."""
    from recsys_amd import dist as D
    from recsys_amd import ops
    from recsys_amd.temp_model.ranker_skelet import ReRankingSystem
    Q, I, K = 4096, args.corpus, 100
    g = torch.Generator(device="cpu").manual_seed(5)
    corpus_full = torch.nn.functional.normalize(torch.randn(I, 128, generator=g), dim=1)
    users = torch.nn.functional.normalize(torch.randn(Q, 128, generator=g), dim=1).to(device)
    lo, hi = rank * I // world, (rank + 1) * I // world
    corpus = corpus_full[lo:hi].to(device)
    del corpus_full
    q0, q1 = rank * Q // world, (rank + 1) * Q // world
    system = ReRankingSystem(None, None, deepfm, {}, corpus)
    buckets = torch.arange(q0, q1, device=device, dtype=torch.int64) % 1000
    last = {}

    def step():
        if world > 1:
            sc, idx = D.retrieve_topk_sharded(users, corpus, lo, K)
            last["cand"] = idx[q0:q1]
            return system.rerank_batch(idx[q0:q1], sc[q0:q1], buckets, final_k=10)
        out = system.recommend_batch(users, buckets, top_k_retrieval=K, final_k=10)
        return out

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    iters = 5
    ops.timing_start()
    t0 = time.perf_counter()
    for _ in range(iters):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=device, dtype=torch.float64)
    if world > 1:
        D.all_reduce_(el, op=torch.distributed.ReduceOp.MAX)
    dt = float(el.item()) / iters
    kt = ops.timing_stop()
    cand = last.get("cand")
    if cand is None:   # one rank: the candidates recommend_batch reranked (same deterministic call)
        cand = ops.retrieve_topk(users, corpus, K)[1]
    n, ms = kt.get("retrieve_topk", (1, 0.0))
    rs = ms / 1e3 / max(n, 1)
    flops = 2.0 * Q * (hi - lo) * 128  # algorithmic (one score per (query, item) of this rank's shard)
    line = {"metric": "retrieve->rerank queries/sec (1M-item corpus, top-100, DeepFM rerank, top-10)",
            "value": round(Q / dt, 1), "unit": "queries/s", "queries": Q, "corpus": I, "n_gpus": world,
            "ms_per_batch": round(dt * 1e3, 3), "rerank_rows_per_s": round(Q * K / dt, 1),
            "data": "synthetic normalised N(0,1) corpus / users, hashed rerank ids",
            "pipeline": "ReRankingSystem.recommend_batch (temp_model/ranker_skelet.py)",
            "retrieval": {"kernel": "rsx_retrieve_topk: topk_bf16_prep_k (corpus bf16 image, cached across calls) + "
                                    "topk_bf16_scan_k (strided sample, best per lane stream) + topk_bf16_thresh_k "
                                    "(per-query threshold) + topk_bf16_collect_k (the one full scan: bf16 MFMA "
                                    "scores, max-gated appends) + topk_bf16_select_k (margin set rescored exactly "
                                    "in fp32, exactness check)",
                          "avg_ms": round(rs * 1e3, 4), "items_per_rank": hi - lo,
                          "achieved_TFLOPs": round(flops / rs / 1e12, 2),
                          "peak_TFLOPs": round(BF16_MFMA_PEAK_TFLOPS, 1),
                          "frac": round(flops / rs / 1e12 / BF16_MFMA_PEAK_TFLOPS, 4),
                          "peak_note": "2 Q I 128 algorithmic FLOPs over the whole op, priced at the dense bf16 "
                                       "MFMA peak (the scan's arithmetic); fp32-MFMA peak 157.3 TF for reference",
                          "corpus_hbm_bytes": int((hi - lo) * 128 * (4 + 2 + 2))}}
    if world > 1:
        coll = "RCCL" if torch.distributed.get_backend() == "nccl" else torch.distributed.get_backend()
        line["sharding"] = (f"corpus by item range ({hi - lo} rows on rank {rank}), per-rank top-{K} with global "
                            f"indices all-gathered over {coll} and merged (score desc, index asc); DeepFM by query "
                            f"({q1 - q0} queries x {K} rows per rank)")
    return line, (out[0], out[2], cand)


def bench_dcn(args, device):
    """The reference's DCN-V2 RankingModel (temp_model/ranker_skelet.py:274-357; SURVEY.md 8f
    #3) scoring 4,096 queries x 100 retrieved candidates (user 128 + item 128 + context 20).
    rows/s with inputs resident in HBM."""
    from recsys_amd.temp_model.ranker_skelet import RankingModel
    R = 4096 * 100
    torch.manual_seed(args.seed)
    model = RankingModel(128, 128, 20).to(device).eval()
    g = torch.Generator(device="cpu").manual_seed(13)
    u = torch.nn.functional.normalize(torch.randn(R, 128, generator=g), dim=1).to(device)
    it = torch.nn.functional.normalize(torch.randn(R, 128, generator=g), dim=1).to(device)
    c = torch.randn(R, 20, generator=g).to(device)
    for _ in range(3):
        model(u, it, c)
    torch.cuda.synchronize()
    iters = 10
    t0 = time.perf_counter()
    for _ in range(iters):
        model(u, it, c)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    return {"metric": "DCN-V2 RankingModel rerank rows/sec (user 128 + item 128 + context 20, 409,600 rows)",
            "value": round(R / dt, 1), "unit": "rows/s", "ms_per_batch": round(dt * 1e3, 4),
            "data": "synthetic normalised vectors, random-init model"}


def bench_hnm(args, device):
    """Hard-negative-mined LogQ loss (inbatch_hnm_corrected_loss_with_stats,
    tower_code/v1_refine_usertower.py:632-692) forward + backward over
    N = 4,096 user rows (one per user of the configs[1] batch), d = 128, 47,063-item table.
    rows/s; the mining kernels (products on the fp32 MFMA + select) timed separately."""
    from recsys_amd import ops
    from recsys_amd.tower_code import v1_refine_usertower as T
    N, I = 4096, 47063
    g = torch.Generator(device="cpu").manual_seed(17)
    W = torch.nn.functional.normalize(torch.randn(I, 128, generator=g), dim=1).to(device).requires_grad_()
    lq = torch.log_softmax(torch.randn(I, generator=g), 0).to(device)
    t = torch.randint(1, I, (N,), generator=g).to(device)
    U = torch.randn(N, 128, generator=g).to(device).requires_grad_()

    def step():
        loss, _ = T.inbatch_hnm_corrected_loss_with_stats(U, W, t, lq)
        loss.backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    iters = 20
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    un = torch.nn.functional.normalize(U.detach(), dim=1)
    itn = torch.nn.functional.normalize(W.detach()[t], dim=1)
    k = int((N - 1) * 0.01)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        ops.hnm_mine(un, itn, t, k, 0.9, 0.1)
    b.record()
    torch.cuda.synchronize()
    mine_ms = a.elapsed_time(b) / iters
    return {"metric": "HNM LogQ loss fwd+bwd rows/sec (inbatch_hnm_corrected_loss_with_stats, N=4096, d=128)",
            "value": round(N / dt, 1), "unit": "rows/s", "ms_per_step": round(dt * 1e3, 4),
            "mining_ms": round(mine_ms, 4), "k": k,
            "mining_tflops_fp32": round(4.0 * N * N * 128 / mine_ms / 1e9, 2),
            "data": "synthetic normalised item table, Gaussian user rows, uniform targets"}


def bench_hard_emphasis(args, device, N=16384):
    """full_batch_hard_emphasis_loss (tower_code/v1_refine_usertower.py:762-822; verdict r5 item 8) forward +
    backward at N = 16,384 rows, d = 128, 47,063-item table: mining (rsx_hnm_mine) + the masked InfoNCE with
    the mined columns' margin (ops.nce_emphasis_loss, no N x N tensor). rows/s, and the same loss in the
    reference's dense form (N x N cosines, emphasis scatter_, masked_fill, F.cross_entropy in torch fp32 on
    this GPU, same mined columns) timed beside it with its peak memory."""
    from recsys_amd.tower_code import v1_refine_usertower as T
    import torch.nn.functional as F
    I = 47063
    g = torch.Generator(device="cpu").manual_seed(23)
    W = F.normalize(torch.randn(I, 128, generator=g), dim=1).to(device).requires_grad_()
    lq = torch.log_softmax(torch.randn(I, generator=g), 0).to(device)
    t = torch.randint(1, I, (N,), generator=g).to(device)
    U = torch.randn(N, 128, generator=g).to(device).requires_grad_()
    tau, margin = 0.1, 0.2

    def step():
        loss, st = T.full_batch_hard_emphasis_loss(U, W, t, lq, temperature=tau, hard_margin=margin)
        loss.backward()
        return loss

    def dense_step():  # the reference's arithmetic on the same mined columns
        u, it = F.normalize(U, dim=1), F.normalize(W[t], dim=1)
        k = max(1, int((N - 1) * 0.01))
        top, _, _ = T.ops.hnm_mine(u.detach(), it.detach(), t, k, 0.9, 1.0)
        logits = (u @ it.T) / tau - lq[t].view(1, -1)
        emph = torch.zeros_like(logits).scatter_(1, top, margin / tau)
        same = t.view(-1, 1) == t.view(1, -1)
        same.fill_diagonal_(False)
        loss = F.cross_entropy((logits + emph).masked_fill(same, float("-inf")), torch.arange(N, device=device))
        loss.backward()
        return loss

    out = {}
    for name, fn in (("native", step), ("dense_torch", dense_step)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        iters = 10
        t0 = time.perf_counter()
        for _ in range(iters):
            loss = fn()
        torch.cuda.synchronize()
        out[name] = {"ms_per_step": round((time.perf_counter() - t0) / iters * 1e3, 4), "loss": round(float(loss), 6),
                     "peak_extra_mem_mb": round((torch.cuda.max_memory_allocated() - base) / 2 ** 20, 1)}
        U.grad = None
        W.grad = None
    dt = out["native"]["ms_per_step"] / 1e3
    return {"metric": f"hard-emphasis loss fwd+bwd rows/sec (full_batch_hard_emphasis_loss, N={N}, d=128)",
            "value": round(N / dt, 1), "unit": "rows/s", "ms_per_step": out["native"]["ms_per_step"],
            "k": max(1, int((N - 1) * 0.01)), "native": out["native"], "reference_form_dense_torch": out["dense_torch"],
            "data": "synthetic normalised item table, Gaussian user rows, uniform targets; tau 0.1, margin 0.2"}


def bench_item_refresh(args, device):
    """refresh-item-vectors (utils/inference_utils.py:74-207) on one GPU: the
    endpoint's eval forward over batches of 4 x 192 = 768 products, d = 128 (the serving
    defaults), bert-base-shaped local BERT, synthetic tokenised products. items/s."""
    import numpy as np
    from recsys_amd import item_tower as IT
    B, R, S = 768, 32, 32
    torch.manual_seed(args.seed)
    model = IT.HybridItemTower(384, 6, 128, 128, bert_model=IT.build_local_bert()).to(device).eval()
    rng = np.random.default_rng(args.seed + 11)
    std = torch.from_numpy(rng.integers(0, 384, (B, 6))).to(device)
    lens = rng.integers(2, R + 1, (B, 9))
    re_mask = torch.from_numpy((np.arange(R)[None, None, :] < lens[..., None]).astype(np.int64)).to(device)
    re_ids = torch.from_numpy(rng.integers(1000, 30521, (B, 9, R))).to(device) * re_mask
    tl = rng.integers(2, S + 1, (B,))
    txt_mask = torch.from_numpy((np.arange(S)[None, :] < tl[:, None]).astype(np.int64)).to(device)
    txt = torch.from_numpy(rng.integers(1000, 30521, (B, S))).to(device) * txt_mask
    with torch.no_grad():
        for _ in range(2):
            model(std, re_ids, re_mask, txt, txt_mask)
        torch.cuda.synchronize()
        iters = 5
        t0 = time.perf_counter()
        for _ in range(iters):
            model(std, re_ids, re_mask, txt, txt_mask)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    return {"metric": "refresh-item-vectors HybridItemTower forward items/sec (batches of 768, d=128, "
                      "bert-base-shaped local BERT)",
            "value": round(B / dt, 1), "unit": "items/s", "ms_per_batch": round(dt * 1e3, 3),
            "data": "synthetic std/RE/text ids, RE field lengths U{2..32}, random BERT weights"}


def bench_item_tower(args, device):
    """BASELINE configs[0] shape on the GPU: HybridItemTower forward (eval) for 256 items,
    d=64, with a locally built bert-base-shaped BERT (random weights). items/s."""
    import numpy as np
    from recsys_amd import item_tower as IT
    B, R, S = 256, 32, 32
    torch.manual_seed(args.seed)
    model = IT.HybridItemTower(384, 6, 64, 128, bert_model=IT.build_local_bert()).to(device).eval()
    rng = np.random.default_rng(args.seed + 7)
    std = torch.from_numpy(rng.integers(0, 384, (B, 6))).to(device)
    lens = rng.integers(2, R + 1, (B, 9))
    re_mask = torch.from_numpy((np.arange(R)[None, None, :] < lens[..., None]).astype(np.int64)).to(device)
    re_ids = torch.from_numpy(rng.integers(1000, 30521, (B, 9, R))).to(device) * re_mask
    tl = rng.integers(2, S + 1, (B,))
    txt_mask = torch.from_numpy((np.arange(S)[None, :] < tl[:, None]).astype(np.int64)).to(device)
    txt = torch.from_numpy(rng.integers(1000, 30521, (B, S))).to(device) * txt_mask
    with torch.no_grad():
        for _ in range(3):
            model(std, re_ids, re_mask, txt, txt_mask)
        torch.cuda.synchronize()
        iters = 10
        t0 = time.perf_counter()
        for _ in range(iters):
            model(std, re_ids, re_mask, txt, txt_mask)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    return {"metric": "HybridItemTower forward items/sec (256 items, d=64, bert-base-shaped local BERT)",
            "value": round(B / dt, 1), "unit": "items/s", "ms_per_batch": round(dt * 1e3, 3),
            "data": "synthetic std/RE/text ids (SURVEY.md 8d config 1), random BERT weights"}, \
        (model, [std, re_ids, re_mask, txt, txt_mask])


def bench_simcse_train(args, device, B=192, iters=3):
    """The item tower's SimCSE training step (item_tower.py:1061-1105; verdict r5 item 6):
    SimCSEModelWrapper(HybridItemTower with a bert-base-shaped local BERT, OptimizedItemTower), two
    views of B synthetic products (the second with 20 % of its RE and text tokens dropped, as
    SimCSERecSysDataset's corruption), symmetric SimCSE loss (fused InfoNCE kernel), backward, AdamW
    with BERT in its own group at lr 1e-5 (:1012-1022). items/s, plus BERT's share of the step: the
    text BERT's forward + backward on the same two views timed alone (HF BertModel under grad, the
    reference's own module), priced at the fp32 MFMA peak (the arithmetic torch runs it in here)."""
    import numpy as np
    from recsys_amd import item_tower as IT
    R, S = 32, 32
    torch.manual_seed(args.seed)
    bert = IT.build_local_bert()
    enc = IT.HybridItemTower(384, 6, 128, 128, bert_model=bert).to(device).train()
    proj = IT.OptimizedItemTower(128, 128).to(device)
    model = IT.SimCSEModelWrapper(enc, proj).train()
    bert_params = [p for n, p in model.named_parameters() if "bert_model" in n]
    other = [p for n, p in model.named_parameters() if "bert_model" not in n]
    opt = torch.optim.AdamW([{"params": bert_params, "lr": 1e-5}, {"params": other, "lr": 1e-3}])
    rng = np.random.default_rng(args.seed + 21)

    def view(drop):
        std = torch.from_numpy(rng.integers(0, 384, (B, 6))).to(device)
        lens = rng.integers(2, R + 1, (B, 9))
        re_mask = (np.arange(R)[None, None, :] < lens[..., None]).astype(np.int64)
        tl = rng.integers(2, S + 1, (B,))
        txt_mask = (np.arange(S)[None, :] < tl[:, None]).astype(np.int64)
        if drop:  # keep [CLS] (position 0) and the first RE token
            re_mask[..., 1:] *= (rng.random((B, 9, R - 1)) >= 0.2)
            txt_mask[:, 1:] *= (rng.random((B, S - 1)) >= 0.2)
        re_ids = torch.from_numpy(rng.integers(1000, 30521, (B, 9, R)) * re_mask).to(device)
        txt = torch.from_numpy(rng.integers(1000, 30521, (B, S)) * txt_mask).to(device)
        return [std, re_ids, torch.from_numpy(re_mask).to(device), txt, torch.from_numpy(txt_mask).to(device)]

    v1 = view(False)
    v2 = [v1[0]] + view(True)[1:]
    for _ in range(2):
        IT.simcse_train_step(model, v1, v2, opt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        loss, _, _ = IT.simcse_train_step(model, v1, v2, opt)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    # the same step with the text BERT through transformers' BertModel (the reference's module) instead
    with IT.bert_train_native(False):
        IT.simcse_train_step(model, v1, v2, opt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            IT.simcse_train_step(model, v1, v2, opt)
        torch.cuda.synchronize()
        dt_hf = (time.perf_counter() - t0) / iters

    # BERT alone: forward + backward of both views' text (the CLS rows' gradient seeded with ones),
    # native packed path (what the step runs) and HF BertModel
    def bert_step(native):
        for v in (v1, v2):
            if native:
                cls = IT.bert_cls_packed_train(bert, v[3], v[4])
            else:
                cls = bert(input_ids=v[3], attention_mask=v[4]).last_hidden_state[:, 0, :]
            cls.sum().backward()

    def timed(native):
        bert_step(native)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            bert_step(native)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters

    assert IT.bert_packed_ok(bert, v1[3], v1[4]) and IT.bert_packed_ok(bert, v2[3], v2[4])
    bt = timed(True)
    bt_hf = timed(False)
    opt.zero_grad(set_to_none=True)
    cfg = bert.config
    Dm, F_, nl = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    lens = torch.cat([v1[4].sum(1), v2[4].sum(1)]).double()
    tok, rows = float(lens.sum()), float(lens.numel())
    attn = 2 * 2 * float((lens * lens).sum()) * Dm  # S = QK^T and O = PV per layer
    # the packed path's forward: every layer's QKV and attention on the valid tokens; out-proj and FFN on
    # every token except in the last layer, which runs them on the [CLS] rows only
    fwd_flops = (nl * (tok * 2 * 3 * Dm * Dm + attn) + (nl - 1) * tok * 2 * (Dm * Dm + 2 * Dm * F_)
                 + rows * 2 * (Dm * Dm + 2 * Dm * F_))
    flops = 3 * fwd_flops  # forward + backward (dX and dW)
    return {"metric": f"SimCSE item-tower train step items/sec (two views, batch {B}, bert-base-shaped local BERT "
                      "fine-tuned, AdamW)",
            "value": round(B / dt, 1), "unit": "items/s", "ms_per_step": round(dt * 1e3, 3), "batch": B,
            "loss": round(float(loss.item()), 5),
            "ms_per_step_with_hf_bertmodel": round(dt_hf * 1e3, 3),
            "bert": {"module": "item_tower.bert_cls_packed_train (packed valid tokens, bf16x3 token GEMMs, varlen "
                               "attention, fused residual+LayerNorm; both views' text, fwd + bwd)",
                     "ms_per_step": round(bt * 1e3, 3), "share_of_step": round(bt / dt, 3),
                     "valid_tokens": int(tok), "padded_tokens": int(2 * B * S),
                     "flops_per_step": int(flops), "achieved_TFLOPs": round(flops / bt / 1e12, 2),
                     "peak_TFLOPs": round(BF16X3_PEAK_TFLOPS, 1), "frac": round(flops / bt / 1e12 / BF16X3_PEAK_TFLOPS, 4),
                     "peak_note": "bf16 dense MFMA 2516.8 TF / 3 split products (the token GEMMs' arithmetic)",
                     "hf_bertmodel_ms_per_step": round(bt_hf * 1e3, 3),
                     "hf_note": "transformers BertModel under grad on the padded [B, S] grid, fp32 (torch's library GEMMs)"},
            "data": "synthetic std / RE / text ids, RE lengths U{2..32}, text lengths U{2..32}, random weights"}


def bench_eval_forward(args, device, model, items, users=4096, iters=10):
    """evaluate_model's tower pass (tower_code/v1_usertower_train.py:548-711 on the GPU:
    SASRecUserTower forward in eval mode, training_mode=False -> the last position's [B, D]
    vector, F.normalize), at 4,096 users of the synthetic H&M-shaped batch, pretrained rows
    gathered on the device. users/s; the model's weights are the headline run's."""
    from recsys_amd import ops, synth
    from recsys_amd.tower_code import v1_usertower_train as TT
    batch = {k: (v.to(device) if torch.is_tensor(v) else v)
             for k, v in synth.make_batch(items, users, seed=args.seed + 300).items()}
    lookup = items.pretrained.to(device)
    kw = {k: batch[k] for k in TT._SEQ_ID_KEYS + TT._STATIC_KEYS}
    was = model.training
    model.eval()

    def step():
        pv = TT.lookup_pretrained(lookup, batch["item_ids"])
        out = model(pretrained_vecs=pv, padding_mask=batch["padding_mask"], training_mode=False, **kw)
        return ops.l2_normalize(out)

    with torch.no_grad():
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            step()
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    model.train(was)
    return {"metric": "evaluate_model tower pass users/sec (SASRecUserTower eval forward, last position, "
                      "4096 users x 50 steps)",
            "value": round(users / dt, 1), "unit": "users/s", "ms_per_batch": round(dt * 1e3, 4),
            "data": "synthetic H&M-shaped batch (dense [B, 50] layout, left-padded), headline weights"}


def train_bench(args, global_batch, steps, warmup, items, cfg, model, item_tower, opt, bucket, rank, world,
                device, sample_clocks=False):
    """Times `steps` full train steps (after `warmup`) on this rank's slice of two seeded global
    batches of `global_batch` users (seeds args.seed + 100, + 101). -> dict with the max-over-ranks
    seconds, per-op HIP-event times, last losses, per-batch valid counts per rank, per-batch distinct
    targets, packed tokens per view, host enqueue time per step and allocator retry counts."""
    from recsys_amd import dist as D
    from recsys_amd import ops, synth
    b_loc = global_batch // world
    lookup = items.pretrained.to(device)
    log_q = item_tower.log_q
    batches = []
    n_dist = []
    for s in range(2):
        g = synth.make_batch(items, global_batch, seed=args.seed + 100 + s)
        # distinct targets of each global batch = the grouped loss's column count
        n_dist.append(int(torch.unique(g["target_ids"][~g["padding_mask"]]).numel()))
        sl = {k: (v[rank * b_loc:(rank + 1) * b_loc] if torch.is_tensor(v) else v) for k, v in g.items()}
        batches.append({k: (v.to(device) if torch.is_tensor(v) else v) for k, v in sl.items()})
    n_valid = [int((~b["padding_mask"]).sum()) for b in batches]
    n_glob = [D.all_gather_counts(n, device) for n in n_valid]
    # packed tokens per view (valid steps + the DuoRec slot of users whose count-1 is a pad)
    n_tok = [int(D.prepare_step_index(b, pretrained_lookup=lookup).packed[0].flat.numel()) for b in batches]
    torch.cuda.synchronize()

    # Each step enqueues its work, then builds the NEXT batch's data-dependent index (packed
    # tokens, grouped targets: the host-synchronising size queries) on a side stream while the
    # GPU runs the step (dist.prepare_step_index_async). Every timed step still builds one index.
    # One rank: the index is built two steps ahead on a background host thread
    # (dist.IndexPrefetcher), so its host synchronisations never hold up the enqueueing of
    # the steps (RSX_PREFETCH_THREAD=0: inline, one step ahead, as with several ranks).
    pending = {}
    enqueue = []
    pf = None
    if world == 1 and not args.no_prefetch_index and os.environ.get("RSX_PREFETCH_THREAD", "1") != "0":
        pf = D.IndexPrefetcher()

    def step(i):
        h0 = time.perf_counter()
        ix = pf.pop(i) if pf is not None else pending.pop(i, None)
        if ix is None:
            ix = D.prepare_step_index(batches[i % 2], pretrained_lookup=lookup)
        out = D.contrastive_step_dp(model, item_tower, log_q, batches[i % 2], opt, cfg, lookup, bucket, index=ix)
        enqueue.append(time.perf_counter() - h0)
        if pf is not None:
            pf.submit(i + 2, batches[i % 2], pretrained_lookup=lookup)
        elif not args.no_prefetch_index:
            pending[i + 1] = D.prepare_step_index_async(batches[(i + 1) % 2], pretrained_lookup=lookup)
        return out

    for i in range(warmup):
        step(i)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    clk0 = gpu_clocks() if sample_clocks else None
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    retries0 = torch.cuda.memory_stats().get("num_alloc_retries", 0)
    enqueue.clear()
    ops.timing_start()
    from recsys_amd import _native as N
    N.lib().rsx_kernel_events(1)  # HIP events around each fused-forward kernel launch (roofline)
    N.lib().rsx_gather_events(1)  # and around each embedding-gather launch (gather roofline)
    t0 = time.perf_counter()
    losses = None
    for i in range(steps):
        losses = step(warmup + i)  # continues the warm-up's step numbering (pending index)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    clk1 = gpu_clocks() if sample_clocks else None
    kernel_times = ops.timing_stop()
    kev = (ctypes.c_float * 256)()
    n_kev = N.lib().rsx_kernel_events_read(kev, 256)
    fwdg_kernel_ms = [float(kev[i]) for i in range(max(n_kev, 0))]
    N.lib().rsx_kernel_events(0)
    gms, gtok = (ctypes.c_float * 256)(), (ctypes.c_int64 * 256)()
    n_gev = N.lib().rsx_gather_events_read(gms, gtok, 256)
    gather_events = [(float(gms[i]), int(gtok[i])) for i in range(max(n_gev, 0))]
    N.lib().rsx_gather_events(0)
    retries = torch.cuda.memory_stats().get("num_alloc_retries", 0) - retries0
    # drain the prefetched indexes of the steps that never ran
    pending.clear()
    if pf is not None:
        pf.close()
    torch.cuda.synchronize()
    # Host cost of one step with the GPU idle when it starts: inside the timed loop the host runs
    # ahead until the launch queue is full, after which every launch waits for the GPU, so the
    # timed loop's enqueue time approaches the GPU step time. Here each step starts from an
    # empty queue; the index is built inline (no prefetch thread), as at world > 1. Untimed.
    unloaded = []
    prof_path = os.environ.get("RSX_HOST_PROFILE")  # cProfile of the unloaded steps (tools only)
    prof = None
    if prof_path:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    trace_path = os.environ.get("RSX_HOST_TRACE")  # torch.profiler CPU table of the same steps (tools only)
    tprof = None
    if trace_path:
        tprof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU],
                                       with_stack=bool(os.environ.get("RSX_HOST_TRACE_STACK")))
        tprof.__enter__()
    for j in range(12 if (prof or tprof) else 3):
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        h0 = time.perf_counter()
        ix = D.prepare_step_index(batches[j % 2], pretrained_lookup=lookup)
        h1 = time.perf_counter()
        D.contrastive_step_dp(model, item_tower, log_q, batches[j % 2], opt, cfg, lookup, bucket, index=ix)
        h2 = time.perf_counter()
        unloaded.append((h1 - h0, h2 - h1))
    torch.cuda.synchronize()
    if prof is not None:
        prof.disable()
        prof.dump_stats(prof_path)
    if tprof is not None:
        tprof.__exit__(None, None, None)
        with open(trace_path, "w") as f:
            f.write(tprof.key_averages().table(sort_by="cpu_time_total", row_limit=120, max_name_column_width=90))
            if os.environ.get("RSX_HOST_TRACE_STACK"):  # where the host copies come from
                for ev in tprof.key_averages(group_by_stack_n=12):
                    if ev.key in ("aten::_to_copy", "aten::copy_", "aten::item", "aten::_local_scalar_dense"):
                        f.write(f"\n{ev.key} calls {ev.count} cpu_total_us {ev.cpu_time_total:.1f}\n  " +
                                "\n  ".join(ev.stack or []) + "\n")
    unloaded = unloaded[1:]
    host_unloaded = {"index_inline_ms": round(1e3 * sum(u[0] for u in unloaded) / len(unloaded), 3),
                     "step_enqueue_ms": round(1e3 * sum(u[1] for u in unloaded) / len(unloaded), 3)}
    host_unloaded["total_ms"] = round(host_unloaded["index_inline_ms"] + host_unloaded["step_enqueue_ms"], 3)
    elapsed = torch.tensor([t1 - t0], device=device, dtype=torch.float64)
    if world > 1:
        D.all_reduce_(elapsed, op=torch.distributed.ReduceOp.MAX)
    return {"elapsed": float(elapsed.item()), "kernel_times": kernel_times, "losses": losses, "n_glob": n_glob,
            "n_dist": n_dist, "n_tok": n_tok, "host_enqueue_ms": round(1e3 * sum(enqueue) / max(len(enqueue), 1), 3),
            "host_unloaded": host_unloaded, "alloc_retries": int(retries), "fwdg_kernel_ms": fwdg_kernel_ms,
            "gather_events": gather_events,
            "clocks": {"before_timed_steps": clk0, "after_timed_steps": clk1} if sample_clocks else None,
            "users_local": b_loc}


def nce_roofline(args, tb, global_batch, rank, world, precision):
    """Roofline of the dominant kernel from the run's own HIP events. bf16x3: the main loss's
    forward fused with the row gradient (nce_grouped_fwdg_x3p_k: S plus the P x B product over
    N_local x D distinct-target columns); fp32: the backward's row-owned pass (S recompute + dU).
    Algorithmic FLOPs per launch = 4 * N_local * D * 128 either way (2 * N * D * d per product;
    SURVEY.md 8d counts 2 N^2 d per product for the ungrouped reference formulation). Peak: the
    MFMA rate of the arithmetic used (fp32 MFMA, or bf16 MFMA / 3 for the bf16x3 split products).
    The timed window is the op's launches (fused kernel + B split + merge) on the launching stream."""
    from recsys_amd import ops
    kernel_times, n_glob, n_dist = tb["kernel_times"], tb["n_glob"], tb["n_dist"]
    flops = 0.0
    for i in range(args.warmup, args.warmup + args.steps):
        flops += 4.0 * n_glob[i % 2][rank] * n_dist[i % 2] * 128
    x3 = precision == "bf16x3"
    h16 = precision == "f16"
    fused = (x3 or h16) and ops._NCE_FUSED_ROWGRAD
    timer = "main/nce_fwd" if fused else "main/nce_bwd_rows"
    launches, ms = kernel_times.get(timer, (0, 0.0))
    op_window_s = (ms / 1e3) / max(launches, 1)
    avg_s = op_window_s
    kms = tb.get("fwdg_kernel_ms") or []
    kernel_only = fused and launches > 0 and len(kms) == launches
    if kernel_only:  # the fused kernel's own launches (events around it alone), not the op window
        avg_s = sum(kms) / len(kms) / 1e3
    achieved = (flops / max(launches, 1)) / avg_s / 1e12 if launches else None
    # f16: the S product is three fp16 MFMAs per product, the gradient product one: two MFMA passes per
    # algorithmic FLOP on average, i.e. the dense fp16 MFMA peak (= bf16's, 2516.8 TF) / 2
    peak = BF16X3_PEAK_TFLOPS if x3 else (F16_SPLIT_PEAK_TFLOPS if h16 else FP32_MFMA_PEAK_TFLOPS)
    traffic, traffic_src, alg_bytes = None, None, None
    if os.path.exists(TRAFFIC_FILE):
        with open(TRAFFIC_FILE) as f:
            tr = json.load(f)
        if (tr.get("precision") == precision and tr.get("global_batch") == global_batch and world == 1 and fused
                and tr.get("partial_slots", 4) == ops._NSPLIT_FWD_GROUPED):
            traffic, traffic_src = tr.get("hbm_bytes_per_launch"), os.path.basename(TRAFFIC_FILE)
            alg_bytes = tr.get("algorithmic_bytes_per_launch")
    fwdg = "nce_grouped_fwdg_x3_k" if os.environ.get("RSX_NCE_FWDG", "1") == "0" else "nce_grouped_fwdg_x3p_k"
    if h16:
        fwdg = f"nce_grouped_fwdg_h_k<{2 if os.environ.get('RSX_NCE_F16_GP') == '2' else 1}>"
    return {"kernel": (f"{fwdg} (main LogQ loss forward fused with the row gradient)"
                       if fused else ("nce_grouped_bwd_x3_k<true>" if x3 else "nce_grouped_bwd_k<true>")
                       + " (main LogQ loss backward, row-owned)"),
            "timer": ("HIP events around each fused-kernel launch (rsx_kernel_events), timed steps"
                      if kernel_only else timer),
            "op_window_ms": round(op_window_s * 1e3, 4), "bound": "mfma",
            "achieved": round(achieved, 2) if achieved else None, "peak": round(peak, 1),
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4) if achieved else None,
            "traffic": traffic, "traffic_source": traffic_src, "algorithmic_bytes": alg_bytes,
            "traffic_over_algorithmic": round(traffic / alg_bytes, 3) if traffic and alg_bytes else None,
            "flops_per_launch": round(flops / max(launches, 1)), "avg_launch_ms": round(avg_s * 1e3, 4),
            "peak_note": ("bf16 dense MFMA 2516.8 TF / 3 split products" if x3 else
                          ("fp16 dense MFMA 2516.8 TF / 2 (logits 3 MFMAs, gradient product 1 per 16-deep step)"
                           if h16 else "fp32-input MFMA dense")),
            "bf16x3_equivalent_frac": (round(achieved / BF16X3_PEAK_TFLOPS, 4) if (h16 and achieved) else None)}


def tower_bytes(T, R, U, layers=2):
    """Algorithmic HBM bytes of one rsx_tower_fwd / rsx_tower_bwd call (csrc/tower.hip, the packed user
    tower of v1_refine_usertower.py:417-510 and its backward): every activation row each launch of the
    program reads and writes once, fp32 (a d-row is 512 B, a QKV row 1,536 B, an FFN row 1,024 B), plus
    8 B of LayerNorm statistics per normed row; weights (< 1 MB per layer) and the step's index arrays
    are not counted. T = packed tokens of both views, R = the tail rows (T/2 + B: the last layer past its
    attention and the head run on those), U = 2B user rows. -> (forward bytes, backward bytes)."""
    d, q, f, st = 512, 1536, 1024, 8
    fwd = 2 * d * T                          # item_proj
    fwd += (2064 + st) * T                   # embedding stage (3 live rows + out + ids) + stats
    fwd += (2 * d + st) * T                  # first norm1
    bwd = 0
    for layer in range(layers):
        P = R if layer == layers - 1 else T  # rows past the attention
        fwd += (d + q) * T + (q + d + 16) * T             # in_proj; attention (+ lse)
        if P != T:
            fwd += 2 * d * P                              # tail: the residual rows gathered
        fwd += (4 * d + st) * P                           # out_proj + residual + norm2
        fwd += (d + 2 * f) * P + (f + d) * P              # FFN1 (gelu' and act), FFN2
        fwd += (4 * d + st) * P if layer < layers - 1 else 3 * d * P  # residual + next norm1 / closing add
        bwd += (5 * d + st) * P if layer < layers - 1 else 2 * d * P  # next norm1 backward / dropout backward
        bwd += (d + 2 * f) * P + (d + f) * P + (f + d) * P + (f + d) * P  # dGELU, dW2, dW1, dX of FFN1
        bwd += (5 * d + st) * P + 2 * d * P + 2 * d * P   # norm2 backward, dX / dW of out_proj
        if P != T:
            bwd += 2 * d * T                              # tail: residual gradient expanded to every row
        bwd += (q + 2 * d + 16 + q) * T                   # attention backward
        bwd += (q + d) * T + (q + d) * T                  # dX / dW of in_proj
    fwd += 2 * d * U + 2 * d * R + (2 * d + st) * R + 2 * d * R + (2 * d + 4) * R  # head (profile, rowadd, LN+GELU, proj, norm)
    bwd += (3 * d + 4) * R + 2 * d * R + 2 * d * R + (3 * d + st) * R + d * R    # head: norm, proj dX/dW, LN+GELU
    bwd += 2 * d * R + 2 * d * R + 4 * d * U                                     # output_proj[0]: dX, dW, profile half
    bwd += (4 * d + st) * T + 3584 * T + 2 * d * T  # first norm1; embedding backward; item_proj dW
    return fwd, bwd


def tower_roofline(tb, steps, warmup):
    """The user tower program's HBM roofline: tower_bytes per launch over the average
    launch time of rsx_tower_fwd / rsx_tower_bwd (HIP events around each native call, timed steps)."""
    kt = tb["kernel_times"]
    out = {}
    T = [2 * n for n in tb["n_tok"]]
    B = tb.get("users_local")
    if not B:
        return None
    for name, idx in (("tower_fwd", 0), ("tower_bwd", 1)):
        n, ms = kt.get(name, (0, 0.0))
        if not n:
            return None
        by = sum(tower_bytes(T[i % 2], T[i % 2] // 2 + B, 2 * B)[idx] for i in range(warmup, warmup + steps)) / steps
        avg = ms / n / 1e3
        out[name] = {"bound": "hbm", "avg_launch_ms": round(avg * 1e3, 4), "algorithmic_bytes": int(by),
                     "bytes_per_packed_token": round(by / (sum(T) / 2), 1),
                     "achieved": round(by / avg / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(by / avg / 1e9 / HBM_PEAK_GBS, 4)}
    tr = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06_tower_traffic_b8192.json")
    if os.path.exists(tr):
        with open(tr) as f:
            t = json.load(f)
        for name in ("tower_fwd", "tower_bwd"):
            if name in t and name in out:
                out[name]["traffic"] = t[name].get("hbm_bytes_per_call")
                out[name]["traffic_source"] = os.path.basename(tr)
    out["model"] = ("bench.tower_bytes: each activation row read / written once per launch of the program, fp32; "
                    "weights and index arrays not counted")
    return out


def gather_roofline(args, tb):
    """Embedding gather (north_star: >= 40 % of HBM): the fused seq-embed forward
    (seq_embed_fwd_k, both dropout views in one packed launch). Algorithmic bytes per token
    (SURVEY.md 8d): 3 live 512-B rows read (projected pretrained row, item-id row, time row; the
    gate-0 tables are skipped), the 512-B output row written, 16 B of ids. NB: the 47k-row item
    table (24 MB) and the 12-row time table are L2/MALL-resident at this size, so this figure
    credits cache hits as HBM bytes; see secondary_gather_1m for DRAM-resident rows."""
    kernel_times, n_tok = tb["kernel_times"], tb["n_tok"]
    ev = tb.get("gather_events") or []
    if ev:  # HIP events around each launch of the gather kernel (issued by the native tower program)
        ms = sum(e[0] for e in ev) / len(ev)
        tok = sum(e[1] for e in ev) / len(ev)
        bpl = 2064.0 * tok
        return {"kernel": "seq_embed_fwd_k", "bound": "hbm", "bytes_per_token": 2064,
                "tokens_per_launch": int(tok), "avg_launch_ms": round(ms, 4), "launches": len(ev),
                "timer": "HIP events around each gather launch inside rsx_tower_fwd (rsx_gather_events), timed steps",
                "achieved": round(bpl / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(bpl / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "cache_note": "item/time tables cache-resident (47k x 512 B + 12 rows); secondary_gather_1m prices "
                              "DRAM-resident rows"}
    g_n, g_ms = kernel_times.get("seq_embed_fwd", (0, 0.0))
    if not g_n:
        return None
    tok = sum(2 * n_tok[i % 2] for i in range(args.warmup, args.warmup + args.steps))  # two views
    bpl = 2064.0 * tok / g_n
    gs = g_ms / 1e3 / g_n
    return {"kernel": "seq_embed_fwd_k", "bound": "hbm", "bytes_per_token": 2064,
            "tokens_per_launch": int(tok / g_n), "avg_launch_ms": round(gs * 1e3, 4),
            "achieved": round(bpl / gs / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(bpl / gs / 1e9 / HBM_PEAK_GBS, 4), "cache_note": "item/time tables cache-resident"}


def train_line(args, tb, global_batch, steps, warmup):
    kt = tb["kernel_times"]
    nf = kt.get("main/nce_fwd", (0, 0.0))
    return {"metric": "SimCSE train-step pairs/sec at d=128 (global batch %d)" % global_batch,
            "value": round(global_batch * steps / tb["elapsed"], 2), "unit": "pairs/s", "steps": steps,
            "warmup": warmup, "ms_per_step": round(1e3 * tb["elapsed"] / steps, 3),
            "valid_positions_per_batch": [sum(c) for c in tb["n_glob"]], "distinct_targets_per_batch": tb["n_dist"],
            "main_loss_fwd_ms": round(nf[1] / max(nf[0], 1), 4), "host_enqueue_ms_per_step": tb["host_enqueue_ms"],
            "host_ms_per_step_unloaded": tb["host_unloaded"], "alloc_retries": tb["alloc_retries"]}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    rank, world, device = setup_dist(args)
    scaling = "strong" if args.batch is not None else "weak"
    if args.batch is None:
        args.batch = args.batch_per_gpu * world
    if args.blas == "rocblas":
        torch.backends.cuda.preferred_blas_library("hipblas")
    elif args.blas == "hipblaslt":
        torch.backends.cuda.preferred_blas_library("hipblaslt")
    elif args.blas == "ck":
        torch.backends.cuda.preferred_blas_library("ck")
    import recsys_amd  # noqa: F401
    from recsys_amd import _native as N
    from recsys_amd import dist as D
    from recsys_amd import ops, synth
    from recsys_amd.tower_code import v1_usertower_train as TT
    from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
    ops.set_nce_precision(args.nce_precision)

    assert args.batch % world == 0, "global batch must divide by the number of GPUs"
    hs = synth.HASH_SIZE
    cfg = TT.PipelineConfig(num_items=args.items, num_prod_types=hs, num_colors=hs, num_graphics=hs,
                            num_sections=hs, dropout=args.dropout)
    items = synth.make_items(num_items=args.items, d=cfg.d_model, seed=args.seed)
    torch.manual_seed(args.seed)
    model = SASRecUserTower(cfg).to(device)
    model.train()
    item_tower = TT.SASRecItemTower(args.items, cfg.d_model, items.log_q.clone()).to(device)
    item_tower.init_from_pretrained(items.pretrained.to(device))
    item_tower.set_freeze_state(args.freeze_items)
    # fused AdamW: one multi-tensor kernel per group instead of the foreach chain (same update)
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay,
                            fused=not args.unfused_adamw)
    if not args.freeze_items:
        opt.add_param_group({"params": list(item_tower.parameters()), "lr": cfg.lr * 0.05})
    bucket = D.GradBucket(list(model.parameters()) + list(item_tower.parameters()))

    # two distinct global batches, this rank's user slice of each, resident in HBM
    tb = train_bench(args, args.batch, args.steps, args.warmup, items, cfg, model, item_tower, opt, bucket, rank,
                     world, device, sample_clocks=(rank == 0))
    total_loss = float(tb["losses"][0].item())
    kt = {k: {"launches": n, "avg_ms": round(t / max(n, 1), 4)} for k, (n, t) in sorted(tb["kernel_times"].items())}
    result = {
        "metric": "SimCSE train-step pairs/sec at d=128, batch %d" % args.batch,
        "value": round(args.batch * args.steps / tb["elapsed"], 2),
        "unit": "pairs/s",
        "n_gpus": world,
        "world_size": (torch.distributed.get_world_size() if world > 1 else 1),
        "collective_backend": (torch.distributed.get_backend() if world > 1 else None),
        "transport": (None if world == 1 else
                      ("RCCL over xGMI" if torch.distributed.get_backend() == "nccl"
                       else f"{torch.distributed.get_backend()} (host-staged; a rehearsal, not an RCCL run)")),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * tb["elapsed"] / args.steps, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": {"f16": "fp32+bf16x3+f16", "bf16x3": "fp32+bf16x3", "fp32": "fp32"}[args.nce_precision],
        "dtype_note": ("fp32 storage and accumulation; token GEMMs bf16x3; grouped LogQ loss (f16): forward logits "
                       "as three fp16 MFMAs of an fp16 hi/lo split (~2^-22 per term), the column pass's as two "
                       "(streamed rows' lo dropped, ~2e-5 on unit vectors: its output is gradients only), gradient "
                       "products as one fp16 MFMA (the reference trains under autocast(float16), "
                       "v1_usertower_train.py:787)"
                       if args.nce_precision == "f16" else None),
        "data": "synthetic (seeded H&M-shaped users/items: sample-calibrated lengths, Zipf(1.0) items; "
                "random-init weights)",
        "config": {"workload": "user-tower two-view contrastive train step (fwd x2 + LogQ in-batch loss + "
                               "DuoRec + bwd + clip + AdamW); N=1: global batch 8192 (BASELINE.json metric); "
                               "weak scaling at 8192 users/GPU, negatives all-gathered over ranks; "
                               "strong_32768 = configs[3] (fixed global batch 32768), retrieve_rerank_sharded = "
                               "configs[4] at N > 1",
                   "users_per_gpu": args.batch // world,
                   "global_batch": args.batch, "seq_len": 50, "d_model": 128, "items": args.items,
                   "valid_positions_per_batch": [sum(c) for c in tb["n_glob"]],
                   "distinct_targets_per_batch": tb["n_dist"], "dropout": args.dropout,
                   "item_matrix": "frozen" if args.freeze_items else "unfrozen (lr x0.05)",
                   "parallelism": f"dp{world} (users split by rank, RCCL all-gather of ids/z, bucketed grad "
                                  f"all-reduce overlapped with backward)",
                   "dense_projection_blas": args.blas, "nce_logit_precision": args.nce_precision},
        "roofline": nce_roofline(args, tb, args.batch, rank, world, args.nce_precision),
        "gather_roofline": gather_roofline(args, tb),
        "tower_roofline": tower_roofline(tb, args.steps, args.warmup),
        "host_enqueue_ms_per_step": tb["host_enqueue_ms"],
        "host_ms_per_step_unloaded": tb["host_unloaded"],
        "alloc_retries": tb["alloc_retries"],
        "kernels": kt,
        "final_loss": round(total_loss, 5),
        "gpu_clocks": tb["clocks"],
        "device": torch.cuda.get_device_name(device),
        "build": N.build_info(),
    }
    del tb
    if world == 1 and not args.no_batch4096 and args.batch != 4096:
        # BASELINE configs[1]: same step, same model and optimiser state, global batch 4096
        t4 = train_bench(args, 4096, args.steps4096, 3, items, cfg, model, item_tower, opt, bucket, rank, world,
                         device)
        result["secondary_batch4096"] = train_line(args, t4, 4096, args.steps4096, 3)
        del t4
        torch.cuda.empty_cache()
    if world == 1 and not args.no_fp32_line:
        # the fp32 parity mode: loss products on the fp32 MFMA, token GEMMs / attention
        # in fp32, at the headline's batch
        prev = (ops.set_nce_precision("fp32"), ops.set_gemm_precision("fp32"), ops.mha_precision())
        ops.set_mha_precision("fp32")
        tf = train_bench(args, args.batch, args.steps_fp32, 2, items, cfg, model, item_tower, opt, bucket, rank,
                         world, device)
        line = train_line(args, tf, args.batch, args.steps_fp32, 2)
        line["metric"] += " [fp32 parity mode: fp32-MFMA loss kernels, fp32 token GEMMs and attention]"
        result["secondary_fp32_mode"] = line
        ops.set_nce_precision(prev[0])
        ops.set_gemm_precision(prev[1])
        ops.set_mha_precision(prev[2])
        del tf
        torch.cuda.empty_cache()
    if not args.no_batch32768 and (world > 1 or args.batch != 32768):
        # configs[3]: FIXED global batch 32,768 (all negatives in one pool), users split by rank
        # (32768 / N each): the strong-scaling line. At N = 1 it is the one-GPU baseline.
        t32 = train_bench(args, 32768, args.steps32768, 2, items, cfg, model, item_tower, opt, bucket, rank, world,
                          device)
        line = train_line(args, t32, 32768, args.steps32768, 2)
        line["metric"] += f" [configs[3]: fixed global batch 32768 on {world} GPU(s), strong scaling]"
        line["n_gpus"] = world
        line["users_per_gpu"] = 32768 // world
        line["scaling"] = "strong"
        del t32
        torch.cuda.empty_cache()
        if world > 1:
            # the 1-GPU baseline of the same global batch in the same run: rank 0 alone (no
            # collectives, dist.local_only) while the other ranks wait at the barrier. Last
            # training line: rank 0's parameters diverge from the others' after it.
            one = None
            if rank == 0:
                with D.local_only():
                    b1 = D.GradBucket([])
                    t1 = train_bench(args, 32768, args.steps32768, 2, items, cfg, model, item_tower, opt, b1, 0, 1,
                                     device)
                one = train_line(args, t1, 32768, args.steps32768, 2)
                del t1
                torch.cuda.empty_cache()
            torch.distributed.barrier()
            if one is not None:
                one["metric"] += " [rank 0 alone, same run: the strong-scaling baseline]"
                line["one_gpu_baseline"] = one
                line["speedup_vs_1gpu"] = round(line["value"] / one["value"], 3)
                line["target_speedup_8gpu"] = 6.0
        result["strong_32768"] = line
        if world == 1:
            result["secondary_batch32768"] = line
    if rank == 0 and world == 1:
        result["secondary_eval_forward"] = bench_eval_forward(args, device, model, items)
        result["secondary_gather_1m"] = bench_gather_1m(device)
        torch.cuda.empty_cache()
    cpu_lines = rank == 0 and world == 1 and not args.no_cpu_baseline
    if rank == 0 and world == 1 and not args.no_deepfm:
        torch.cuda.empty_cache()
        deepfm, result["secondary"], dfm_x = bench_deepfm(args, device)
        if not args.no_rerank:
            result["secondary_retrieve_rerank"], rr_out = bench_retrieve_rerank(args, device, deepfm)
            result["secondary_dcn_rerank"] = bench_dcn(args, device)
        if cpu_lines:
            dst = deepfm_cpu_state(deepfm)
            line = result["secondary"]
            with torch.no_grad():
                dfm_logits = deepfm.forward_logits(dfm_x)[0].float().cpu()
            line["cpu_baseline"] = cpu_baseline_deepfm(args, dst, dfm_x, dfm_logits)
            line["gpu_over_cpu"] = round(line["value"] / line["cpu_baseline"]["value"], 1)
            if not args.no_rerank:
                line = result["secondary_retrieve_rerank"]
                line["cpu_baseline"] = cpu_baseline_retrieve_rerank(args, dst, rr_out)
                line["gpu_over_cpu"] = round(line["value"] / line["cpu_baseline"]["value"], 1)
            del dst
        del deepfm, dfm_x
        torch.cuda.empty_cache()
    if world > 1 and not args.no_deepfm and not args.no_rerank:
        # configs[4] on N GPUs: corpus sharded by item range, DeepFM rerank sharded by query
        from recsys_amd.temp_model.ranker_skelet import DeepFM
        torch.cuda.empty_cache()
        torch.manual_seed(args.seed + 3)       # the replicated reranker: identical on every rank
        deepfm = DeepFM([args.deepfm_vocab] * 39, device=device)
        result["retrieve_rerank_sharded"], _ = bench_retrieve_rerank(args, device, deepfm, rank, world)
        del deepfm
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_item_tower:
        result["secondary_item_tower"], (it_model, it_inputs) = bench_item_tower(args, device)
        if cpu_lines:
            line = result["secondary_item_tower"]
            line["cpu_baseline"] = cpu_baseline_item_tower(args, it_model, it_inputs)
            line["gpu_over_cpu"] = round(line["value"] / line["cpu_baseline"]["value"], 1)
        del it_model, it_inputs
        result["secondary_item_refresh"] = bench_item_refresh(args, device)
        result["secondary_simcse_train"] = [bench_simcse_train(args, device, B) for B in (192, 768)]
        result["secondary_hard_emphasis"] = bench_hard_emphasis(args, device)
        torch.cuda.empty_cache()
        result["secondary_hnm"] = bench_hnm(args, device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, items, cfg, args.batch, args.seed + 100, device)
        result["gpu_over_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
        if "secondary_batch4096" in result:       # configs[1]: the same step at 4,096 users
            line = result["secondary_batch4096"]
            line["cpu_baseline"] = cpu_baseline(args, items, cfg, 4096, args.seed + 100, device)
            line["gpu_over_cpu"] = round(line["value"] / line["cpu_baseline"]["value"], 1)
        if "strong_32768" in result:
            result["strong_32768"]["cpu_baseline"] = None
            result["strong_32768"]["cpu_baseline_note"] = (
                "not timed: the oracle step at 32,768 users (N ~ 600k valid steps) is ~16x the headline's "
                "N x N loss work, i.e. ~40 min on these cores, past BASELINE.md's bounded-sample rule; the "
                "headline and configs[1] lines carry the measured per-pair CPU rate")
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
