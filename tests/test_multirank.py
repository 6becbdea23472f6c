"""The N>1 path on CPU (gloo, world_size 2): the film-tile sharding contract
and bench.py's distributed plumbing.

Each rank owns the 16x16 tiles t with t % world == rank
(mtsg_render_params.tile_stride / tile_offset), renders them
into a full-size ImageBlock (the oracle stands in for the GPU here: same
ownership rule, counter-mode RNG), and the blocks are summed.  The sum must
equal the single-rank render -- the same property the GPU parity test
`test_tiling_is_additive` checks on the device.  bench.py's
dist_setup / barrier / max_over_ranks / gather_frame run exactly as under
torch.distributed.run, and `bench.py --gpus N` refuses to start N ranks on
fewer visible GPUs.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import torch.multiprocessing as mp

from conftest import REPO, SCENES


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import sys
    for p in (os.path.join(REPO, "my-mitsuba_amd"), REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch
    import bench
    import mtsg
    from oracle import pyoracle as O

    r, w, local, pg = bench.dist_setup(world)
    assert (r, w, local) == (rank, world, rank)
    scene = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {"width": 72, "height": 40, "spp": 4})
    p = scene.params(max_depth=6)
    p.tile_stride = world
    p.tile_offset = rank
    block, st = O.render(scene.desc, p, scene.border, rng=O.RNG_COUNTER, threads=2)
    t = torch.from_numpy(block.copy())   # all_reduce works in place
    bench.barrier(pg)
    pg.all_reduce(t)                    # host-side additive gather (ImageBlock::put)
    m = bench.max_over_ranks(pg, float(rank + 1))
    # bench.py's gather: rank 0 sends per-tile windows (as mtsg_render_device_tiles
    # returns them), rank 1 a block of the whole rectangle
    part = ("win", tile_windows(scene, p, world, rank)) if rank == 0 else ("block", block)
    frame = bench.gather_frame(pg, rank, world, part, 72, 40, scene.border)
    ids = bench.all_gather_obj(pg, f"dev{rank}", world)
    assert ids == [f"dev{r}" for r in range(world)]
    if rank == 0:
        np.save(os.path.join(out_dir, "sum.npy"), t.numpy())
        np.save(os.path.join(out_dir, "frame.npy"), frame)
        np.save(os.path.join(out_dir, "max.npy"), np.array([m]))
        np.save(os.path.join(out_dir, "samples0.npy"), np.array([st.samples]))
    else:
        assert frame is None
    pg.destroy_process_group()


def tile_windows(scene, p, stride, offset):
    """The per-tile ImageBlocks (16 + 2 border square) of the tiles of deal key
    offset + v * stride, each rendered alone by the oracle and cut out of its
    block: the layout mtsg_render_device_tiles writes."""
    from oracle import pyoracle as O
    tiles_x, tiles_y = (p.tile_w + 15) // 16, (p.tile_h + 15) // 16
    b = scene.border
    win = 16 + 2 * b
    keys = range(offset, tiles_x * tiles_y, stride)
    out = np.zeros((len(keys), win, win, 5), np.float32)
    q = p.copy()
    q.tile_stride = tiles_x * tiles_y
    for v, key in enumerate(keys):
        q.tile_offset = key
        block, _ = O.render(scene.desc, q, b, rng=O.RNG_COUNTER, threads=2)
        ty = key // tiles_x
        tx = (key % tiles_x + ty) % tiles_x
        h, w = min(win, block.shape[0] - 16 * ty), min(win, block.shape[1] - 16 * tx)
        out[v, :h, :w] = block[16 * ty:16 * ty + h, 16 * tx:16 * tx + w]
    return out


def test_two_rank_tile_sharding_sums_to_full_frame(tmp_path):
    import mtsg
    from oracle import pyoracle as O
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    scene = mtsg.Scene(os.path.join(SCENES, "cbox.xml"), {"width": 72, "height": 40, "spp": 4})
    p = scene.params(max_depth=6)
    full, st = O.render(scene.desc, p, scene.border, rng=O.RNG_COUNTER, threads=2)
    summed = np.load(tmp_path / "sum.npy")
    assert np.load(tmp_path / "max.npy")[0] == 2.0
    # 72x40 -> 5x3 = 15 tiles (ragged last column and row); rank 0 owns the
    # tiles of even deal key ty * 5 + (tx - ty) mod 5 (include/mtsg.h)
    own0 = sum(min(16, 72 - 16 * tx) * min(16, 40 - 16 * ty) for ty in range(3) for tx in range(5)
               if (ty * 5 + (tx - ty) % 5) % 2 == 0)
    assert own0 != sum(min(16, 72 - 16 * (t % 5)) * min(16, 40 - 16 * (t // 5)) for t in range(0, 15, 2))
    assert np.load(tmp_path / "samples0.npy")[0] == own0 * 4
    keys = mtsg.tile_deal_keys(72, 40)
    assert keys[0, 16] == 1 and keys[16, 0] == 9 and keys[16, 16] == 5   # (tx, ty) = (1, 0), (0, 1), (1, 1)
    assert full[..., 4].sum() > 0
    np.testing.assert_allclose(summed, full, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(np.load(tmp_path / "frame.npy"), full, rtol=1e-5, atol=1e-6)


def test_bench_refuses_more_ranks_than_gpus():
    """`bench.py --gpus 2` without a launcher starts the ranks itself, but not on
    fewer visible GPUs than ranks (here: none) unless --allow-shared is given;
    it fails loudly before any rank starts."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env={**os.environ, "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode != 0
    assert "refusing" in r.stderr and "--allow-shared" in r.stderr, r.stderr[-2000:]
    assert r.stdout.strip() == ""
