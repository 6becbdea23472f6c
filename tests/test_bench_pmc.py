"""bench.py quotes PMC counters (roofline.traffic, tcc_hit_rate, per-kernel
GB/s) only from a committed set collected on the same kernel instantiation
and configuration (a two-level line once carried the flattened
kernel's traffic)."""
import argparse
import json

import bench


def args(**kw):
    a = dict(workload="bunny15", instancing="flatten", kd_build="host", width=1280, height=720, spp=256,
             emulate_ranks=0, batch_paths=0, finish_paths=-1, balance_rounds=4)
    a.update(kw)
    return argparse.Namespace(**a)


def test_trace_kernel_names():
    assert bench.trace_kernel(args()) == "k_trace_s<false, 16, false, false>"
    assert bench.trace_kernel(args(instancing="two-level")) == "k_trace_s<false, 16, true, false>"


def test_lookup_matches_the_whole_key_only(tmp_path):
    flat = bench.pmc_key(args())
    two = bench.pmc_key(args(instancing="two-level"))
    dev = bench.pmc_key(args(kd_build="device"))
    share = bench.pmc_key(args(emulate_ranks=8))
    batch = bench.pmc_key(args(batch_paths=1 << 28))     # other launches: other counters
    finish = bench.pmc_key(args(finish_paths=0))
    build = dict(flat, build="0123456789abcdef")          # counters of another libmtsg.so
    assert flat["build"] == bench.device_build_id() and flat["build"]
    assert len({json.dumps(k, sort_keys=True) for k in (flat, two, dev, share, batch, finish, build)}) == 7
    (tmp_path / "r03_pmc_c3.json").write_text(json.dumps({"key": flat, "kernels": {"k_trace_s<false, 16, false, false>": {}}}))
    (tmp_path / "r02_pmc_c3.json").write_text(json.dumps({"key": flat, "kernels": {"old": {}}}))
    j, src = bench.pmc_lookup(flat, str(tmp_path))
    assert src.endswith("r03_pmc_c3.json") and "k_trace_s<false, 16, false, false>" in j["kernels"]
    for k in (two, dev, share, batch, finish, build):
        assert bench.pmc_lookup(k, str(tmp_path)) == (None, None)


def test_rocprof_names_normalise_to_the_instantiation():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "pmc_kernels", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "pmc_kernels.py"))
    pk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pk)
    n = pk.kernel_name
    assert n("void (anonymous namespace)::k_trace_s<false, 16, false>(mtsg::DevScene, mtsg::DevPaths, int, int, "
             "unsigned int, unsigned long long*)") == "k_trace_s<false, 16, false>"
    assert n("void (anonymous namespace)::k_trace_s<false, 16, true, false>(mtsg::DevScene)") == "k_trace_s<false, 16, true, false>"
    assert n("(anonymous namespace)::k_camera(mtsg::DevCamera, mtsg::DevIntegrator)") == "k_camera"
    assert n("void (anonymous namespace)::k_splat<5, 4>(mtsg::DevCamera, float*, int, int)") == "k_splat<5, 4>"


def test_pmc_sets_are_per_frame():
    """a PMC pass renders only the frames it is normalised by
    (bench.py --pmc-pass), so a committed set's k_shade time per frame (rocprof
    average x launches per frame) agrees with the HIP-event figure of the bench
    line of the same configuration -- the multi-step 1/8-share set too."""
    import glob
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pairs = {"c3": "bunny15", "c4_share8": "c4_e8", "c5": "c5", "c3_two_level": "bunny15_two_level"}
    checked = 0
    for tag, bench_tag in pairs.items():
        sets = sorted(glob.glob(os.path.join(repo, "profiles", f"r*_pmc_{tag}.json")))
        if not sets:
            continue
        pj = json.load(open(sets[-1]))
        if "frames_fetch_pass" not in pj:
            continue   # sets of round 5 and before: not normalised per frame, never quoted
        rnd = os.path.basename(sets[-1]).split("_")[0]
        line = os.path.join(repo, "profiles", f"{rnd}_bench_{bench_tag}.json")
        if not os.path.exists(line):
            continue
        b = json.load(open(line))
        ks = [v for n, v in pj["kernels"].items() if n.startswith("k_shade<") and "rocprof_ms_per_frame" in v]
        pmc_ms = sum(v["rocprof_ms_per_frame"] for v in ks)
        hip_ms = b["kernels"]["shade_ms"]
        assert abs(pmc_ms - hip_ms) <= 0.10 * hip_ms, (tag, pmc_ms, hip_ms)
        # and the bench line quotes the set's per-frame bytes for k_shade
        assert abs(b["kernels"]["pmc"]["k_shade"]["rocprof_ms_per_frame"] - pmc_ms) < 2e-3
        checked += 1
    assert checked >= 1 or not glob.glob(os.path.join(repo, "profiles", "r06_pmc_*.json"))


def test_scheduling_and_tree_options_key_their_own_sets():
    # options that change the launches (the tree, the tail kernel's shading
    # group, lanes) key their own sets; their defaults keep the plain key, so
    # the committed sets stay quotable by a default run
    base = bench.pmc_key(args())
    assert bench.pmc_key(args(kd_props="", finish_shade_min=0, lanes=0, stagger=-1)) == base
    others = [bench.pmc_key(args(kd_props="kdStopPrims=5")), bench.pmc_key(args(finish_shade_min=1)),
              bench.pmc_key(args(lanes=2)), bench.pmc_key(args(stagger=2))]
    for k in others:
        assert k != base
        assert {n: v for n, v in k.items() if n in base} == base   # only the option's own entry differs
