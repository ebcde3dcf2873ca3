#!/usr/bin/env python3
"""Layout-search throughput: score_layouts (mobile_env.scoring; chooseBaseStation.ipynb's
qoeValue for a whole batch) on N MComCustom layouts (randint(5, 10) stations, 7 UEs,
velocity 10, one 20-step episode each), on the GPU.

Prints one JSON line: the end-to-end score_layouts wall time (engine build, device seeding,
the episode, scores to the host) and the episode alone (20 fused steps with per-env layouts,
per-episode QoE statistics), both as layouts/s and env-steps/s.

usage: python tools/bench_scoring.py [--layouts 100000] [--repeats 5]"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mobile-env-gan_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layouts", type=int, default=100000)
    ap.add_argument("--repeats", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from mobile_env.collect import draw_layouts
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.scoring import layout_scores, score_layouts

    N = args.layouts
    xy, cnt = draw_layouts(random.Random(0), N)
    dev = torch.device("cuda", 0)
    score_layouts(xy[:1024], cnt[:1024], device=dev)  # warm (module load, first launches)
    torch.cuda.synchronize(dev)
    e2e_all = []
    for _ in range(3):  # (one-shot timings of engine build + run vary with the host: best of 3)
        t0 = time.perf_counter()
        out = score_layouts(xy, cnt, device=dev)
        e2e_all.append(time.perf_counter() - t0)
    e2e = min(e2e_all)

    # the episode alone: 20 fused steps on a prepared engine, QoE statistics accumulated
    p = EngineParams(num_envs=N, num_ues=7, num_bs=xy.shape[1], velocity=10.0)
    eng = StepEngine(p, xy, np.full(N, 2024), bs_count=cnt, device=dev, qoe_stats=True)
    eng.reset()
    eng.step(20)
    torch.cuda.synchronize(dev)
    times = []
    for _ in range(args.repeats):
        eng.reset()
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        eng.step(20)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - a)
    sc = layout_scores(eng.qoe_stats)["Score"].cpu().numpy()
    assert np.allclose(sc, out["Score"], rtol=1e-12, equal_nan=True)
    eng.close()
    ep = min(times)
    print(json.dumps({
        "bench": "score_layouts", "layouts": N, "ues": 7, "steps_per_episode": 20,
        "end_to_end_s": e2e, "end_to_end_s_all": e2e_all, "layouts_per_s_end_to_end": N / e2e,
        "episode_s_best": ep, "episode_s_all": times,
        "layouts_per_s_episode": N / ep, "env_steps_per_s_episode": N * 20 / ep,
        "best_layout": int(out["best"]), "best_score": float(out["Score"][out["best"]])}))


if __name__ == "__main__":
    main()
