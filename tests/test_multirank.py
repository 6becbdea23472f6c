"""The N>1 path on CPU (gloo, world_size 2): the film-tile sharding contract
and bench.py's distributed plumbing.

Each rank owns the 16x16 tiles t with t % world == rank
(mtsg_render_params.tile_stride / tile_offset), renders them
into a full-size ImageBlock (the oracle stands in for the GPU here: same
ownership rule, counter-mode RNG), and the blocks are summed.  The sum must
equal the single-rank render -- the same property the GPU parity test
`test_tiling_is_additive` checks on the device.  bench.py's
dist_setup / barrier / max_over_ranks run exactly as under torch.distributed.run.
"""
import os
import socket

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
    t = torch.from_numpy(np.ascontiguousarray(block))
    bench.barrier(pg)
    pg.all_reduce(t)                    # host-side additive gather (ImageBlock::put)
    m = bench.max_over_ranks(pg, float(rank + 1))
    if rank == 0:
        np.save(os.path.join(out_dir, "sum.npy"), t.numpy())
        np.save(os.path.join(out_dir, "max.npy"), np.array([m]))
        np.save(os.path.join(out_dir, "samples0.npy"), np.array([st.samples]))
    pg.destroy_process_group()


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
