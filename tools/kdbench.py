#!/usr/bin/env python3
"""The reference's kd-tree benchmark (src/tests/test_kd.cpp:86-131) on the GPU:
data/tests/bunny.ply alone, 10M chords between two uniform points of the
bounding sphere ((-0.016840, 0.110154, -0.001537), r = 0.2), each an any-hit
query with mint 0 and no maxt (ShapeKDTree::rayIntersect(const Ray &)), three
iterations, "MRays/s" and the fraction of rays that hit.  The GPU answers
through mtsg_trace_shadow (host buffers: the wall time includes the PCIe
copies; the kernel time comes from rocprofv3 when run under it).  The CPU
oracle answers the same rays on one thread (the reference benchmark's loop)
and on all cores, and the answers must agree.
usage: python tools/kdbench.py [n_rays] [iterations]"""
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "my-mitsuba_amd"))
sys.path.insert(0, REPO)
import mtsg  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

CENTER = np.array([-0.016840, 0.110154, -0.001537], np.float64)
RADIUS = 0.2


def sphere_points(rng, n):
    # warp::squareToUniformSphere (warp.cpp): z = 1 - 2u, phi = 2 pi v
    u, v = rng.random(n), rng.random(n)
    z = 1.0 - 2.0 * u
    r = np.sqrt(np.maximum(0.0, 1.0 - z * z))
    phi = 2.0 * np.pi * v
    return np.stack([r * np.cos(phi), r * np.sin(phi), z], 1)


def chords(n, seed):
    rng = np.random.default_rng(seed)
    p1 = CENTER + sphere_points(rng, n) * RADIUS
    p2 = CENTER + sphere_points(rng, n) * RADIUS
    d = p2 - p1
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = p1
    rays[:, 3:6] = d
    rays[:, 6] = 0.0
    rays[:, 7] = np.inf
    return rays


def scene():
    # the bunny alone, with an environment emitter (no geometry) so the scene loads
    xml = f"""<scene version="0.5.0">
  <integrator type="path"/>
  <sensor type="perspective"><film type="hdrfilm"><integer name="width" value="8"/><integer name="height" value="8"/></film></sensor>
  <shape type="ply"><string name="filename" value="{REPO}/scenes/bunny.ply"/><bsdf type="diffuse"/></shape>
  <emitter type="envmap"><string name="filename" value="{REPO}/scenes/sky512.pfm"/></emitter>
</scene>"""
    fd, path = tempfile.mkstemp(suffix=".xml")
    with os.fdopen(fd, "w") as f:
        f.write(xml)
    try:
        return mtsg.Scene(path)
    finally:
        os.unlink(path)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    s = scene()
    g = mtsg.GPUScene(s, 0)
    out = {"benchmark": "test_kd.cpp:86-131 bunny chords (any-hit, mint 0, maxt inf)", "rays": n,
           "triangles": int(s.info.n_triangles), "gpu": [], "cpu": {}}
    g.trace_shadow(chords(1 << 16, 99))   # warm-up
    for j in range(iters):
        rays = chords(n, j)
        t0 = time.perf_counter()
        occ = g.trace_shadow(rays)
        dt = time.perf_counter() - t0
        out["gpu"].append({"iteration": j, "hit_fraction": round(float(occ.mean()), 5),
                           "wall_ms": round(dt * 1e3, 2), "wall_mrays_s": round(n / dt / 1e6, 1)})
        print(f"GPU iteration {j}: {occ.mean() * 100:.3f}% hit, {dt * 1e3:.1f} ms wall (PCIe included) "
              f"-> {n / dt / 1e6:.1f} MRays/s", flush=True)
    # the CPU oracle on a bounded sample, and parity on it
    m = min(n, 1_000_000)
    rays = chords(m, 0)
    t0 = time.perf_counter()
    occ_c1 = O.trace_shadow(s.desc, rays, threads=1)
    t1 = time.perf_counter() - t0
    from bench import cgroup_cpus
    quota = cgroup_cpus()
    cores = max(1, min(os.cpu_count() or 1, int(quota + 0.999))) if quota else (os.cpu_count() or 1)
    t0 = time.perf_counter()
    occ_cn = O.trace_shadow(s.desc, rays, threads=cores)
    tn = time.perf_counter() - t0
    occ_g = g.trace_shadow(rays)
    agree = float((occ_g == occ_c1).mean())
    assert np.array_equal(occ_c1, occ_cn)
    out["cpu"] = {"rays": m, "one_thread_mrays_s": round(m / t1 / 1e6, 2), "all_threads_mrays_s": round(m / tn / 1e6, 2),
                  "threads": cores, "hit_fraction": round(float(occ_c1.mean()), 5)}
    out["parity"] = {"rays": m, "agreement": agree}
    print(f"CPU oracle: {m / t1 / 1e6:.2f} MRays/s on 1 thread, {m / tn / 1e6:.2f} on all threads; "
          f"GPU/oracle agreement {agree:.6f}", flush=True)
    print(json.dumps(out))
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "kdbench.json"), "w") as f:
        json.dump(out, f, indent=1)
    g.close()
    assert agree > 0.9999


if __name__ == "__main__":
    main()
