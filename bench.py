"""Headline benchmark: images/sec of one ViT-B/16 CLIP+MAE training step
(BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W
  (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Workload per GPU = BASELINE.json configs[2] / configs[3]: ViT-B/16 @224, 256
images per GPU, MAE mask 0.75 + 8-layer 512-d decoder, 6-layer frozen
DistilBERT text tower (T=25), soft-target CLIP loss over the GLOBAL batch
(embeddings all-gathered), fused AdamW -- forward + backward + optimizer every
step, bf16 MFMA with fp32 master weights. Synthetic inputs already resident in
HBM (uint8 pixels ImageNet-normalised, input_ids randint(5,300)).
Weak scaling: per-GPU batch fixed, value = global images / max-over-ranks time.

Extra fields: "roofline" (the launch shape with the largest total time per
step -- forward / dgrad GEMMs and the grouped weight-gradient launches of the
main stream -- timed live during the timed steps on its stream),
"roofline_fwd_dgrad" (the same for the largest forward / dgrad GEMM shape),
"cpu_baseline" (the CPU oracle of /oracle on a bounded sample, rank 0 at N=1
only), "loss_delta_vs_ref" (C0 fp32 parity), "u8_input_pipeline" (N=1: the
step with the uint8 pixel H2D copy inside the timed region, main.py:55).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0    # MI355X dense fp8 (block-scaled e4m3) MFMA
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E (MI355X_MICROARCH.md; 6.3 TB/s measured copy)
PEAK_F32_TFLOPS = 157.3
IMG_FLOPS_C2 = 60.2e9       # algorithmic FLOP / image, SURVEY.md §8d / Appendix C

# BASELINE.json configs by SURVEY.md §8 label. The driver's default line is C2
# (N=1) / C3 (N>1: the same 256 images per GPU, global batch 256*N).
CONFIGS = {
    "c2": dict(model=dict(model_name="vit_base_patch16_224", size=224, image_embedding=768, mask_ratio=0.75),
               batch=256, flops=60.2e9,
               workload="C2/C3: ViT-B/16 224 MAE(0.75)+CLIP, 8x512 decoder, DistilBERT-6 frozen T=25, AdamW, "
                        "bf16 MFMA / fp32 master"),
    "c1": dict(model=dict(model_name="vit_base_patch16_224", size=224, image_embedding=768, mask_ratio=0.0),
               batch=256, flops=107.3e9,
               workload="C1: ViT-B/16 224 CLIP-only (mask 0, the reference's path), DistilBERT-6 frozen T=25, "
                        "AdamW, bf16 MFMA / fp32 master"),
    "c4": dict(model=dict(model_name="vit_large_patch14_336", size=336, image_embedding=1024, mask_ratio=0.75),
               batch=128, flops=376.4e9,
               workload="C4: ViT-L/14 336 MAE(0.75)+CLIP, 8x512 decoder, DistilBERT-6 frozen T=25, AdamW, "
                        "fp32 master"),
}


def synthetic_batch(B, S, T, seed, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    px = torch.randint(0, 256, (B, 3, S, S), generator=g, dtype=torch.uint8).to(device)
    mean = torch.tensor([0.485, 0.456, 0.406], device=device).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=device).view(1, 3, 1, 1)
    img = ((px.float() / 255.0) - mean) / std
    ids = torch.randint(5, 300, (B, T), generator=g).to(device)
    am = torch.ones(B, T, dtype=torch.int64, device=device)
    return {"image": img.contiguous(), "input_ids": ids, "attention_mask": am}


def build_model(cfg_over):
    from mae_clip_amd import config as CFG
    for k, v in cfg_over.items():
        setattr(CFG, k, v)
    from mae_clip_amd.CLIP import CLIPModel
    return CLIPModel()


def parity_c0(device):
    """|loss(product, fp32 parity mode) - loss(CPU oracle, fp64)| at C0 (ViT-Tiny @32,
    2-layer text, mask .75, B=8) -- the 'loss delta vs ref' of the metric."""
    sys.path.insert(0, ROOT)
    from tests.helpers import build_pair, make_batch
    prod, ref = build_pair("fp32")
    prod.eval()
    ref.eval()
    b = make_batch(8, 32)
    with torch.no_grad():
        lp = prod({k: v.to(device) for k, v in b.items()}).item()
        lr = ref(dict(b, image=b["image"].double())).item()
    return abs(lp - lr), lp, lr


def parity_headline(device, precision="bf16", B=4):
    """|loss(product) - loss(CPU oracle, fp64)| at the metric's own model shapes
    and precision: ViT-B/16 @224, mask .75, 8x512 decoder, 6-layer text (the C2
    step this bench times), bf16, B=4 (the oracle is a CPU fp64 restatement of
    CLIP.py:34-43 + modules.py, so B is kept small), forward in eval mode."""
    sys.path.insert(0, ROOT)
    from tests.helpers import build_pair, make_batch
    kw = dict(model_name="vit_base_patch16_224", size=224, image_embedding=768, text_layers=6, mask_ratio=0.75,
              decoder_embed_dim=512, decoder_depth=8, decoder_num_heads=16)
    prod, ref = build_pair(precision, **kw)
    prod.eval()
    ref.eval()
    b = make_batch(B, 224, seed=12)
    with torch.no_grad():
        lp = prod({k: v.to(device) for k, v in b.items()}).item()
        lr = ref(dict(b, image=b["image"].double())).item()
    return abs(lp - lr), abs(lp - lr) / max(1.0, abs(lr)), lp, lr


def train_curve_headline(device, precision="bf16", B=4, steps=5):
    """The reference's train loop at the metric's model shapes vs the fp64 CPU
    oracle (tests/helpers.py train_curve; asserted by
    tests/test_model_gpu.py test_vitb_c2_train_curve_vs_oracle)."""
    sys.path.insert(0, ROOT)
    from tests.helpers import train_curve
    return train_curve(device, precision, B, steps)


def cpu_model_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(seconds_budget=20.0):
    """The CPU oracle (pure torch fp32, same ops as the reference) on a bounded
    sample of the same workload: ViT-B/16 MAE+CLIP, 6-layer text, B=16.
    Threads = the job's CPU share (OMP_NUM_THREADS, 16 on the GPU box; the
    box's os.cpu_count() is the whole host's, several jobs share it)."""
    from oracle.ref_model import CLIPModel as RefCLIP, OracleConfig
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cfg = OracleConfig(model_name="vit_base_patch16_224", img_size=224, text_layers=6, mask_ratio=0.75,
                       decoder_dim=512, decoder_depth=8, decoder_heads=16)
    torch.manual_seed(0)
    m = RefCLIP(cfg)
    m.train()
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
    B = 16
    batch = synthetic_batch(B, 224, 25, 0, "cpu")
    times = []
    t_start = time.perf_counter()
    for i in range(4):
        t0 = time.perf_counter()
        opt.zero_grad()
        loss = m(batch)
        loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > seconds_budget and i >= 1:
            break
    timed = times[1:] if len(times) > 1 else times
    per_step = sorted(timed)[len(timed) // 2]
    return {"value": B / per_step, "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model_name(),
            "calibration": "profiles/r02/cpu_calibration.json",
            "sample": f"oracle ViT-B/16 MAE+CLIP + 6-layer text, fp32 CPU, B={B}, median of {len(timed)} "
                      f"step(s) after 1 warm-up (fwd+bwd+AdamW)"}


def pmc_traffic(key):
    """HBM bytes per launch of GEMM shape `key` from the committed rocprofv3 PMC
    summaries (profiles/*/traffic_*.json, written by tools/pmc_traffic.sh:
    FETCH_SIZE x 2 + WRITE_SIZE, separate passes, MI355X_MICROARCH.md §HBM).
    PMC counters cannot be read inside a timed run, so the matching file of the
    newest round directory (profiles/rNN, then the file name) is reported with
    its path; None when no summary covers the shape."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic_*.json"))):
        try:
            r = json.load(open(f))
        except (OSError, ValueError):
            continue
        if r.get("shape", "").split(">")[0] == key.split(">")[0]:
            best = (f, r)   # sorted paths: a later round's file wins
    if best is None:
        return None, None
    return best[1]["hbm_bytes"], os.path.relpath(best[0], ROOT)


class KernelTimer:
    """Brackets GEMM launches with HIP events on the launching stream; reports
    the shape with the largest total time.

    Eager steps: one HIP event pair per launch. Under HIP-graph capture
    torch-ROCm refuses event-record nodes ("External events are disallowed in
    rocm"), so the launch is bracketed by two 1-lane timestamp kernels on the
    same stream (maeclip_timestamp: s_memrealtime, 100 MHz) that are captured
    with it; every replay re-times it, snapshot() queues a device copy of the
    spans right after the replay's launch (no host sync between steps) and
    harvest() reads them all after the timed loop."""

    def __init__(self):
        self.records = {}
        self.active = False
        self.only = None     # timed region: bracket only this key's launches
        self.captured = []   # (key, flops, slot) bracketed inside the graph
        self.ts = None       # device int64 [2 * slots] timestamps
        self.snaps = []      # per timed replay: device copies of ts
        self.limit = {}      # key -> most launches bracketed per captured step

    def hook(self, key, flops, nbytes, launch):
        if not self.active:
            return launch()
        from mae_clip_amd.functions import side_stream, microbatch_active
        if torch.cuda.current_stream() == side_stream(torch.device("cuda", torch.cuda.current_device())):
            # side-stream launches (text tower, weight gradients) overlap the
            # main chain by design: their event spans are not kernel durations
            return launch()
        mb = microbatch_active()
        if mb is not None:
            # micro-batch chains (functions.MicroBatches) run concurrently: only
            # micro-batch 0's launches (current stream) are bracketed, and their
            # spans include the other chain's co-running kernels (key tagged)
            if mb > 0:
                return launch()
            key = key + " [2 concurrent micro-batches]"
        # the timed region brackets only the shapes picked from the warm step,
        # whose keys carry the tags above
        if self.only is not None and key not in self.only:
            return launch()
        if torch.cuda.is_current_stream_capturing():
            from mae_clip_amd import _lib
            lib, st = _lib.lib(), torch.cuda.current_stream().cuda_stream
            if self.ts is None:
                self.ts = torch.zeros(2 * 64, dtype=torch.int64, device="cuda")
            i = len(self.captured)
            if i >= 64 or sum(1 for c in self.captured if c[0] == key) >= self.limit.get(key, 64):
                return launch()
            _lib.check(lib.maeclip_timestamp(self.ts.data_ptr() + 16 * i, st), "maeclip_timestamp")
            launch()
            _lib.check(lib.maeclip_timestamp(self.ts.data_ptr() + 16 * i + 8, st), "maeclip_timestamp")
            self.captured.append((key, flops, nbytes, i))
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        self.records.setdefault(key, [flops, nbytes, []])[2].append((s, e))

    def snapshot(self):
        """Right after a replay is launched: queue a device copy of its
        timestamps (stream-ordered after the replay, no host sync), so the
        timed loop's host turnaround between steps carries no D2H read."""
        if self.captured:
            from mae_clip_amd import kernels as K
            self.snaps.append(K.copy_words(self.ts, torch.empty_like(self.ts)))

    def harvest(self):
        """After the timed loop: add the captured launches' durations (ms) of
        every snapshot (one D2H copy for the whole run)."""
        snaps, self.snaps = self.snaps, []
        if not self.captured or not snaps:
            return
        from mae_clip_amd import _lib
        khz = float(_lib.lib().maeclip_wallclock_khz()) or 100000.0
        for t in torch.stack(snaps).cpu():
            t = t.view(-1, 2)
            for key, flops, nbytes, i in self.captured:
                self.records.setdefault(key, [flops, nbytes, []])[2].append(float(t[i, 1] - t[i, 0]) / khz)

    def table(self, steps, file):
        rows = []
        for key, (flops, nbytes, evs) in self.records.items():
            ms = [x if isinstance(x, float) else x[0].elapsed_time(x[1]) for x in evs]
            avg = sum(ms) / len(ms)
            rows.append((sum(ms) / steps, len(ms) / steps, flops / avg / 1e9, nbytes / avg / 1e6, key))
        rows.sort(reverse=True)
        print(f"GEMM total {sum(r[0] for r in rows):.3f} ms/step", file=file)
        for t, n, tf, gbs, key in rows:
            print(f"{t:8.3f} ms/step {n:5.1f} launches/step {tf:7.1f} TF/s {gbs:7.1f} GB/s  {key}", file=file)

    def summary(self, pred=None):
        """(key, flops, total ms, launches, bytes) of the launch shape with the
        largest total time, among the keys pred accepts (default: all)."""
        best = None
        for key, (flops, nbytes, evs) in self.records.items():
            if pred is not None and not pred(key):
                continue
            ms = [x if isinstance(x, float) else x[0].elapsed_time(x[1]) for x in evs]
            tot = sum(ms)
            if best is None or tot > best[2]:
                best = (key, flops, tot, len(ms), nbytes)
        return best


def is_fwd_dgrad(key):
    """forward / dgrad GEMM shapes (not the grouped weight-gradient launches)"""
    return not key.startswith("wgrad_grouped")


def is_alone(key):
    """launches that run alone on the GPU (no co-running micro-batch chain):
    their span is the kernel's own duration"""
    return "concurrent" not in key


def roofline(best, img_flops, batch, ms, precision):
    """roofline object of one launch shape (bench JSON contract): achieved =
    algorithmic bytes (HBM-bound) or FLOPs (MFMA-bound) per launch / measured
    average launch duration; bound picked by arithmetic intensity vs the ridge."""
    key, flops, tot_ms, nl, nbytes = best
    avg_s = tot_ms / nl / 1000.0
    tf = flops / avg_s / 1e12
    gbs = nbytes / avg_s / 1e9
    mpeak = PEAK_FP8_TFLOPS if " fp8" in key else PEAK_BF16_TFLOPS
    ai = flops / nbytes
    ridge = mpeak * 1e12 / (PEAK_HBM_GBS * 1e9)
    traffic, tsrc = pmc_traffic(key)
    if ai >= ridge:
        bound, ach, peak, unit = "mfma", tf, mpeak, "TFLOP/s"
    else:
        bound, ach, peak, unit = "hbm", gbs, PEAK_HBM_GBS, "GB/s"
    kind = "grouped weight-gradient GEMM " if key.startswith("wgrad_grouped") else "gemm "
    r = {"bound": bound, "kernel": kind + key, "achieved": round(ach, 1), "peak": peak, "unit": unit,
         "frac": round(ach / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
         "traffic_source": tsrc, "algorithmic_bytes": nbytes, "flops": flops,
         "arith_intensity": round(ai, 1), "ridge": round(ridge, 1),
         "tflops": round(tf, 1), "mfma_frac": round(tf / mpeak, 4), "gbs": round(gbs, 1),
         "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
         "avg_launch_us": round(avg_s * 1e6, 1), "launches": nl}
    if "concurrent" in key:
        r["span"] = ("micro-batch 0's launch while micro-batch 1's chain co-runs on the other stream: "
                     "the span includes the co-running kernels, so it is an upper bound on the kernel's "
                     "own duration (the kernel trace in profiles/ has that)")
    if img_flops:
        stf = img_flops * batch / (ms / 1000.0) / 1e12
        r.update(step_tflops=round(stf, 1), step_frac=round(stf / PEAK_BF16_TFLOPS, 4),
                 step_frac_peak="bf16 dense 2.5 PF/s")
        if precision == "fp8":
            r.update(step_frac_fp8=round(stf / PEAK_FP8_TFLOPS, 4), step_frac_fp8_peak="fp8 dense 5.0 PF/s")
    return r


def standalone_gemm(key, device, reps=20):
    """The launch shape `key` ("M.. N.. K.. <A><B> epi<e> <in>><out>", the keys
    kernels.gemm gives LAUNCH_HOOK) run ALONE on the GPU on fresh tensors: the
    median of `reps` HIP-event spans of single launches on the current stream,
    i.e. the kernel's own duration (a span taken inside the step includes the
    other micro-batch chain's co-running kernels). Returns (us, plan note)."""
    import re
    from mae_clip_amd import kernels as K
    m = re.match(r"M(\d+) N(\d+) K(\d+) ([KR])([KR]) epi(\d+) (\w+)>(\w+)", key)
    if m is None or m.group(7) != "bf16":
        return None
    M, N, Kd = int(m.group(1)), int(m.group(2)), int(m.group(3))
    la, lb, epi = "KR".index(m.group(4)), "KR".index(m.group(5)), int(m.group(6))
    odt = torch.bfloat16 if m.group(8) == "bf16" else torch.float32
    g = torch.Generator(device=device).manual_seed(7)
    A = (torch.randn((M, Kd) if la == 0 else (Kd, M), generator=g, device=device) * 0.5).to(torch.bfloat16)
    B = (torch.randn((N, Kd) if lb == 0 else (Kd, N), generator=g, device=device) * 0.5).to(torch.bfloat16)
    C = torch.empty(M, N, device=device, dtype=odt)
    kw = {}
    if epi in (K.EPI_GELU, K.EPI_GELU_D):
        kw = dict(aux_out=torch.empty(M, N, device=device, dtype=torch.bfloat16), ldaux=N,
                  bias=torch.randn(N, generator=g, device=device))
    elif epi in (K.EPI_DGELU, K.EPI_MUL_AUX):
        kw = dict(aux=torch.randn(M, N, generator=g, device=device).to(torch.bfloat16), ldaux=N)
    elif epi == K.EPI_RESID:
        kw = dict(resid=torch.randn(M, N, generator=g, device=device), ldr=N,
                  bias=torch.randn(N, generator=g, device=device))
    fn = lambda: K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, la, lb, epilogue=epi, **kw)
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    us = sorted(s.elapsed_time(e) * 1e3 for s, e in ts)[reps // 2]
    return us


def u8_leg(model, opt, args, size, device, use_graph):
    """The reference's per-step input hop (main.py:55 copies the batch to the
    GPU) timed INSIDE the step: the decoded uint8 RGB pixels [B, S, S, 3] sit in
    pinned host memory, each step copies them (and the text ids / mask) to the
    device asynchronously and the step normalises them inside the patch gather
    and the MAE target read (A.Normalize + permute fused, dataset.py:49, :34).
    A second CapturedStep on the same model / optimizer; reported beside the
    headline (whose inputs are HBM-resident), never as `value`."""
    from mae_clip_amd.graph import CapturedStep
    g = torch.Generator(device="cpu").manual_seed(2000)
    B, T = args.batch, 25
    host = {"image": torch.randint(0, 256, (B, size, size, 3), generator=g, dtype=torch.uint8).pin_memory(),
            "input_ids": torch.randint(5, 300, (B, T), generator=g).pin_memory(),
            "attention_mask": torch.ones(B, T, dtype=torch.int64).pin_memory()}
    runner = CapturedStep(model, opt, enabled=use_graph, eager_steps=2)

    def step():
        if runner.static is not None:
            for k, v in host.items():
                runner.static[k].copy_(v, non_blocking=True)
            return runner.step(runner.static)
        return runner.step({k: v.to(device, non_blocking=True) for k, v in host.items()})

    for _ in range(3):
        step().item()
    torch.cuda.synchronize()
    steps = max(1, min(args.steps, 10))
    t0 = time.perf_counter()
    for i in range(steps):
        step()
        if i > 0 and not args.sync_loss:
            runner.previous_loss()   # step i-1's loss, read while step i runs (as in the headline loop)
        elif args.sync_loss:
            runner.loss_value()
    runner.loss_value()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # the whole drop-in loop of main.py:54-66: the input copy of :55 AND the
    # blocking loss read of :64 before the next step is queued
    t0 = time.perf_counter()
    for i in range(steps):
        step()
        runner.loss_value()
    torch.cuda.synchronize()
    el_drop = time.perf_counter() - t0
    h2d = sum(v.numel() * v.element_size() for v in host.values())
    return {"value": round(B * steps / el, 2), "unit": "images/s", "ms_per_step": round(el / steps * 1e3, 3),
            "steps": steps, "h2d_bytes_per_step": h2d,
            "h2d_bytes_per_step_fp32_reference": B * 3 * size * size * 4 + 2 * B * T * 8,
            "what": "uint8 HWC pixels + text ids/mask copied host(pinned)->device inside every timed step "
                    "(main.py:55), A.Normalize/permute fused into the patch gather and MAE target read",
            "drop_in_loop": {"value": round(B * steps / el_drop, 2), "unit": "images/s",
                             "ms_per_step": round(el_drop / steps * 1e3, 3),
                             "what": "the same copy inside every step plus each step's loss read (blocking) "
                                     "before the next is queued: main.py:55 and :64 together"}}


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N ranks through
    torch.distributed.run (one process per GPU) and relay rank 0's JSON line.
    The parent never touches the GPU (no HIP context before the children)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="BASELINE.json config (SURVEY.md §8 labels); the default line is C2/C3")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default: the config's)")
    ap.add_argument("--mask-ratio", type=float, default=None)
    ap.add_argument("--precision", choices=["bf16", "fp8"], default="bf16",
                    help="GEMM operand precision (fp8: OCP e4m3 forward and dgrad GEMMs of the encoder and decoder stacks "
                         "(config.fp8_grad_format), e8m0 per-32 blocks / per-row scales on the activations, "
                         "per-channel on the weights)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--sync-loss", action="store_true",
                    help="read each step's loss before queueing the next (default: once the next step is queued)")
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of one HIP graph per step")
    ap.add_argument("--gemm-table", action="store_true", help="per-shape GEMM times to stderr")
    ap.add_argument("--dp", action="store_true",
                    help="data-parallel code path (RCCL process group, gathers, grad all-reduce) even at N=1")
    ap.add_argument("--no-side-stream", action="store_true",
                    help="text tower and weight gradients on the main stream (config.side_stream = False)")
    ap.add_argument("--microbatches", type=int, default=None,
                    help="samples of each bf16 transformer stack split into this many concurrent chains "
                         "(config.stack_microbatches; default: the config's)")
    ap.add_argument("--no-u8-leg", action="store_true",
                    help="skip the extra input-pipeline measurement (uint8 pixels H2D + fused Normalize in the step)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the launcher started WORLD_SIZE="
                         f"{os.environ.get('WORLD_SIZE')} ranks")
    # the driver reads ONE JSON line from stdout: route everything else written
    # to fd 1 (RCCL's version banner, library chatter) to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    use_dp = world > 1 or args.dp
    if use_dp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group("nccl", device_id=device, rank=rank, world_size=world)

    from mae_clip_amd import kernels as K
    from mae_clip_amd.optim import AdamW
    from mae_clip_amd.distributed import DataParallel
    from mae_clip_amd.graph import CapturedStep

    cfg = CONFIGS[args.config]
    if args.batch is None:
        args.batch = cfg["batch"]
    mcfg = dict(cfg["model"])
    if args.mask_ratio is not None:
        mcfg["mask_ratio"] = args.mask_ratio
    args.mask_ratio = mcfg["mask_ratio"]
    img_flops = cfg["flops"] if args.mask_ratio == cfg["model"]["mask_ratio"] else None
    size = mcfg["size"]
    model = build_model(dict(mcfg, text_layers=6, decoder_embed_dim=512, decoder_depth=8,
                             decoder_num_heads=16, precision=args.precision,
                             side_stream=not args.no_side_stream,
                             **({} if args.microbatches is None else {"stack_microbatches": args.microbatches}))).to(device)
    model.train()
    dp = DataParallel(model) if use_dp else None
    opt = AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
    batch = synthetic_batch(args.batch, size, 25, 1000 + rank, device)

    timer = KernelTimer()
    if not args.no_kernel_timer:
        K.LAUNCH_HOOK = timer.hook

    # one HIP graph per step (mae_clip_amd.graph): steps 1-2 eager, step 3
    # captured, then replays -- at N=1 and, with the RCCL collectives captured
    # inside the graph, at N>1. --gemm-table stays eager.
    use_graph = not args.no_graph and not args.gemm_table
    runner = CapturedStep(model, opt, enabled=use_graph, eager_steps=2, dp=dp)
    use_graph = runner.enabled
    warmup = max(args.warmup, 3) if use_graph else max(args.warmup, 2)

    def step():
        # after capture the graph's static input buffers ARE the batch
        # (synthetic inputs resident in HBM): no per-step copy
        return runner.step(runner.static if runner.static is not None else batch)

    # warm-up: time every GEMM launch of the second (eager, warm) step to find
    # the dominant shape; afterwards only that shape's launches are bracketed
    # (~8 per step instead of ~250; in graph mode the brackets are captured
    # with the step at i == 2 and re-timed by every replay)
    for i in range(warmup):
        timer.active = (i == 1) or args.gemm_table or (use_graph and i == 2)
        loss = step()
        loss.item()
        if i == 1 and timer.records and not args.gemm_table:
            # bracket the dominant launch shape overall (incl. the grouped
            # weight gradients) and the dominant forward / dgrad GEMM shape
            k_alone, k_fd = (timer.summary(is_alone) or timer.summary())[0], timer.summary(is_fwd_dgrad)[0]
            timer.only = {k_alone, k_fd}
            if k_fd != k_alone:
                # two bracketed launches per step of the forward / dgrad shape: the
                # timestamp kernels sit in that micro-batch chain's critical path
                timer.limit[k_fd] = 2
            timer.records = {}
    torch.cuda.synchronize()
    timer.records = {}
    if use_dp:
        dist.barrier()
    torch.cuda.synchronize()
    timer.active = True
    t0 = time.perf_counter()
    losses = []
    for i in range(args.steps):
        loss = step()
        timer.snapshot()
        # main.py:64 reads the loss every step; here step k's value (published by
        # the step into mapped host memory, no copy launch) is read once step k + 1
        # is queued, so the host's turnaround does not idle the GPU between steps
        # (--sync-loss: read each step's own loss before queueing the next)
        if args.sync_loss:
            losses.append(runner.loss_value())
        elif i > 0:
            losses.append(runner.previous_loss())
    if not args.sync_loss:
        losses.append(runner.loss_value())   # the last step's, after it finished
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    assert len(losses) == args.steps and all(math.isfinite(v) for v in losses), losses
    timer.harvest()
    timer.active = False
    # the drop-in loop as main.py:64 runs it: each step's loss read (blocking)
    # before the next step is queued; reported beside the headline, not as value
    sync_el = None
    if not args.sync_loss:
        if use_dp:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steps):
            step()
            assert math.isfinite(runner.loss_value())
        torch.cuda.synchronize()
        sync_el = time.perf_counter() - t1
    if use_dp:
        dist.barrier()
        t = torch.tensor([elapsed, sync_el or 0.0], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t[0].item()
        sync_el = t[1].item() if sync_el is not None else None
    global_batch = args.batch * world
    value = global_batch * args.steps / elapsed
    ms = elapsed / args.steps * 1000.0

    if rank == 0 and args.gemm_table and not args.no_kernel_timer:
        timer.table(args.steps, sys.stderr)
    u8 = None
    if not args.no_u8_leg and world == 1:
        u8 = u8_leg(model, opt, args, size, device, use_graph)
    if rank == 0:
        roof = roof2 = None
        # the dominant launch among those that run alone (a co-running
        # micro-batch chain would make its span more than its own duration)
        best = (timer.summary(is_alone) or timer.summary()) if not args.no_kernel_timer else None
        if best is not None:
            roof = roofline(best, img_flops, args.batch, ms, args.precision)
            best2 = timer.summary(is_fwd_dgrad)
            if best2 is not None and best2[0] != best[0]:
                roof2 = roofline(best2, img_flops, args.batch, ms, args.precision)
                # the same shape alone on the GPU: the kernel's own duration
                # (the in-step span includes the co-running micro-batch chain)
                try:
                    us = standalone_gemm(best2[0].split(" [")[0], device)
                except Exception as e:   # reported, never hides the perf line
                    us, roof2["standalone_error"] = None, repr(e)
                if us:
                    key2, flops2, _, _, nbytes2 = best2
                    alone = roofline((key2.split(" [")[0], flops2, us / 1000.0, 1, nbytes2), 0, args.batch, ms,
                                     args.precision)
                    roof2["standalone"] = {k: alone[k] for k in ("achieved", "frac", "avg_launch_us", "tflops",
                                                                 "mfma_frac", "gbs", "hbm_frac")}
                    roof2["standalone"]["what"] = ("median of 20 single launches of this shape alone on the GPU "
                                                   "(fresh tensors, HIP events), after the timed loop")
        metric = ("images/sec/node ViT-B/16 CLIP+MAE step" if args.config != "c4"
                  else "images/sec/node ViT-L/14@336 CLIP+MAE step")
        out = {"metric": metric, "value": round(value, 2), "unit": "images/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
               "data": "synthetic (uint8 pixels ImageNet-normalised, input_ids randint(5,300)), random-init weights",
               "config": {"workload": cfg["workload"].replace("fp32 master", f"{args.precision} MFMA / fp32 master")
                          if args.config == "c4" else cfg["workload"], "label": args.config.upper(),
                          "global_batch": global_batch, "per_gpu_batch": args.batch, "image_size": size,
                          "mask_ratio": args.mask_ratio, "parallelism": f"dp{world}",
                          "img_flops": img_flops},
               "loss": round(loss.item(), 4), "roofline": roof, "roofline_fwd_dgrad": roof2,
               "u8_input_pipeline": u8,
               "loss_read": ("sync: each step's loss read before the next step is queued (main.py:64)"
                             if args.sync_loss else
                             "pipelined: step k's loss (published by the step into mapped host memory) read right "
                             "after step k+1 is queued; every step's loss is read"),
               "sync_loss_leg": None if sync_el is None else {
                   "value": round(global_batch * args.steps / sync_el, 2), "unit": "images/s",
                   "ms_per_step": round(sync_el / args.steps * 1000.0, 3), "steps": args.steps,
                   "what": "the same captured step, each step's loss read (blocking) before the next is queued, "
                           "as main.py:64's loss.item() does"},
               "step_mode": "hip-graph" if use_graph else "eager",
               "rccl": {"backend": dist.get_backend(), "world_size": dist.get_world_size()} if use_dp else None}
        if world == 1 and not args.no_parity:
            try:
                dl, lp, lr = parity_c0(device)
                out["loss_delta_vs_ref"] = {"abs": dl, "product": lp, "oracle": lr,
                                            "config": "C0 ViT-Tiny/16@32, 2-layer text, mask .75, B=8, fp32"}
            except Exception as e:  # reported, never hides the perf line
                out["loss_delta_vs_ref"] = {"error": repr(e)}
            if args.config == "c2":
                try:
                    t0 = time.time()
                    da, dr, lp, lr = parity_headline(device, args.precision)
                    out["loss_delta_vs_ref_headline"] = {
                        "abs": da, "rel": dr, "product": lp, "oracle": lr, "precision": args.precision,
                        "config": "C2 model shapes (ViT-B/16@224, mask .75, 8x512 decoder, 6-layer text), B=4, "
                                  "eval-mode forward vs the fp64 CPU oracle", "seconds": round(time.time() - t0, 1)}
                except Exception as e:
                    out["loss_delta_vs_ref_headline"] = {"error": repr(e)}
                try:
                    t0 = time.time()
                    out["train_curve_vs_ref_headline"] = dict(train_curve_headline(device, args.precision),
                                                              seconds=round(time.time() - t0, 1))
                except Exception as e:
                    out["train_curve_vs_ref_headline"] = {"error": repr(e)}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if use_dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
