"""Multi-rank path on CPU: world_size 2 (and 3) over gloo.  Each rank renders its interleaved
rows with the host build of the kernel logic, the tiles are gathered to rank 0 and un-permuted,
and the result must equal a single-process render bit for bit (the Philox stream is keyed by the
global pixel index).  Only rank 0 holds the frame."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, row_block, out_path):
    import sys
    for p in (ROOT, os.path.join(ROOT, "tests", "kernel_emu")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import emu
    from raytrace_amd import scenes
    from raytrace_amd.dist import ShardedRenderer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cs, scene, seed = scenes.cornell_box(spp=4, width=40)

    def tile_fn(settings, w, s, n, r, rb):
        return emu.render(settings, w, s, n_shards=n, shard=r, row_block=rb, nthreads=2)

    sr = ShardedRenderer(cs, scene, row_block=row_block, tile_fn=tile_fn)
    img = sr.render(seed)
    if rank == 0:
        np.save(out_path, img)
    else:
        assert img is None and sr.gathered is None  # the gather's destination is rank 0 alone
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,row_block", [(2, 4), (3, 3), (2, 1)])
def test_sharded_render_equals_single_render(emu_mod, tmp_path, world, row_block):
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), row_block, out), nprocs=world, join=True)
    got = np.load(out)
    from raytrace_amd import scenes
    cs, scene, seed = scenes.cornell_box(spp=4, width=40)
    full = emu_mod.render(cs, scene, seed)
    assert got.shape == full.shape == (40, 40, 3)
    np.testing.assert_array_equal(got, full)


def test_shard_row_partition_covers_every_row_once():
    from raytrace_amd.ray import shard_row_index, shard_rows
    for h, n, rb in [(600, 8, 4), (338, 3, 4), (1, 4, 1), (675, 7, 5)]:
        rows = np.concatenate([shard_row_index(h, n, r, rb) for r in range(n)])
        real = rows[rows < h]
        assert sorted(real.tolist()) == list(range(h))
        assert all(len(shard_row_index(h, n, r, rb)) == shard_rows(h, n, rb) for r in range(n))
