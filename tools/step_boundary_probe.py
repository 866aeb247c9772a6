"""Step-boundary probe (no profiler): how long the GPU idles between two
replays of the captured C2 step.

Two device timestamps (maeclip_timestamp, the REALTIME counter) are captured
with the step: one before the model's first launch, one after the loss is
published. After every replay a copy of both is queued (maeclip_copy_f32, no
host sync). gap_k = start_{k+1} - end_k is the idle time at the boundary
(it includes the 4-B copy launch and whatever the runtime queues at a graph
launch); dur_k = end_k - start_k is the step's own GPU span.

    python tools/step_boundary_probe.py [--steps 40] [--read prev|none|sync] [--config c2]

Prints one JSON line. Env knobs of the HIP runtime are taken as they are (the
probe is run under each setting by tools/gpu_r3.sh step 'boundary')."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--read", default="prev", choices=["prev", "none", "sync"])
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()

    import bench
    from mae_clip_amd import _lib
    from mae_clip_amd import kernels as K
    from mae_clip_amd.optim import AdamW
    from mae_clip_amd.graph import CapturedStep

    device = torch.device("cuda", 0)
    cfg = bench.CONFIGS[args.config]
    mcfg = dict(cfg["model"])
    model = bench.build_model(dict(mcfg, text_layers=6, decoder_embed_dim=512, decoder_depth=8,
                                   decoder_num_heads=16, precision="bf16", side_stream=True)).to(device)
    model.train()
    opt = AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
    batch = bench.synthetic_batch(cfg["batch"], mcfg["size"], 25, 1000, device)

    lib = _lib.lib()
    ts = torch.zeros(2, dtype=torch.int64, device=device)

    def stamp(i):
        _lib.check(lib.maeclip_timestamp(ts.data_ptr() + 8 * i, torch.cuda.current_stream().cuda_stream),
                   "maeclip_timestamp")

    fwd = model.forward

    def fwd_stamped(*a, **kw):
        stamp(0)
        return fwd(*a, **kw)

    model.forward = fwd_stamped
    runner = CapturedStep(model, opt, enabled=True, eager_steps=2)
    pub = runner._publish

    def pub_stamped(loss):
        pub(loss)
        stamp(1)

    runner._publish = pub_stamped

    def step():
        return runner.step(runner.static if runner.static is not None else batch)

    for _ in range(max(args.warmup, 3)):
        step().item()
    torch.cuda.synchronize()
    snaps = torch.zeros(args.steps, 2, dtype=torch.int64, device=device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
        K.copy_words(ts, snaps[i])
        if args.read == "sync":
            runner.loss_value()
        elif args.read == "prev" and i > 0:
            runner.previous_loss()
    runner.loss_value()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    khz = float(lib.maeclip_wallclock_khz()) or 100000.0
    s = snaps.cpu().double() / khz   # ms
    dur = (s[:, 1] - s[:, 0]).tolist()
    gap = (s[1:, 0] - s[:-1, 1]).tolist()

    def med(v):
        v = sorted(v)
        return v[len(v) // 2]

    env = {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_HIP", "DEBUG_CLR", "HIP_FORCE", "GPU_MAX"))}
    print(json.dumps({"probe": "step_boundary", "config": args.config, "read": args.read, "env": env,
                      "steps": args.steps, "ms_per_step_wall": round(el / args.steps * 1e3, 3),
                      "img_per_s": round(cfg["batch"] * args.steps / el, 1),
                      "gpu_span_ms_median": round(med(dur), 3), "gap_ms_median": round(med(gap), 4),
                      "gap_ms_max": round(max(gap), 4), "gap_ms_min": round(min(gap), 4),
                      "gap_ms_mean": round(sum(gap) / len(gap), 4)}), flush=True)


if __name__ == "__main__":
    main()
