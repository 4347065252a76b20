"""Multi-GPU rendering: one process per GPU, rows dealt to ranks, framebuffer gathered to rank 0
over RCCL.

Pixels are independent (Ray.hs:238) and the Philox stream is keyed by the GLOBAL pixel index,
so any row partition renders exactly the image a single GPU renders.  Rank r owns the rows
{y : (y / row_block) % world_size == r} (interleaved blocks balance the uneven per-row cost of
a scene); every rank's tile has the same padded row count, so the exchange is one gather of
equal-size tiles to rank 0 (torch.distributed.gather: RCCL point-to-point sends into
rank 0's frame, 0.9 MB per rank at 600x600 on 8 GPUs, each over its own xGMI link) — the only
collective on the path.  Only rank 0 holds the frame; it un-permutes the rows.

`tile_fn` lets the CPU tests drive the same partition / gather / assembly logic over `gloo`
with a host renderer; the product path renders on the local GPU through DeviceScene.
"""
from __future__ import annotations

import numpy as np

from .camera import CameraSettings, image_height
from .ray import DeviceScene, assemble_shards, shard_rows


class ShardedRenderer:
    def __init__(self, settings: CameraSettings, world, row_block: int = 4, device=None, tile_fn=None, group=None,
                 precision: str = "f64"):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.group = group
        self.settings = settings
        self.row_block = row_block
        self.world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.h = image_height(settings)
        self.w = int(settings.cs_imageWidth)
        self.rows = shard_rows(self.h, self.world_size, row_block)
        self.tile_fn = tile_fn
        self.precision = precision
        dtype = torch.float64 if precision == "f64" else torch.float32
        if tile_fn is None:
            self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
            self.scene = DeviceScene(world, device=self.device.index or 0)
        else:
            self.device = torch.device("cpu")
            self.scene = None
            self.world = world
        self.tile = torch.empty((self.rows, self.w, 3), dtype=dtype, device=self.device)
        # the frame: rank 0 only (a gather's destination); the tiles land in consecutive row blocks
        self.gathered = (torch.empty((self.world_size * self.rows, self.w, 3), dtype=dtype, device=self.device)
                         if self.rank == 0 else None)

    def render_tile(self, seed, stream=None):
        """Enqueue (GPU) or compute (tile_fn) this rank's rows into self.tile."""
        if self.tile_fn is not None:
            self.tile.copy_(self.torch.from_numpy(np.ascontiguousarray(
                self.tile_fn(self.settings, self.world, seed, self.world_size, self.rank, self.row_block))).to(
                self.tile.dtype))
            return
        s = stream if stream is not None else self.torch.cuda.current_stream(self.device)
        self.scene.render_async(self.settings, seed, self.tile.data_ptr(), s.cuda_stream, n_shards=self.world_size,
                                shard=self.rank, row_block=self.row_block, precision=self.precision)

    def gather(self, async_op=False):
        """Every rank's tile into rank 0's frame (views of it: no copy after the receive)."""
        if self.world_size > 1:
            parts = list(self.gathered.chunk(self.world_size)) if self.rank == 0 else None
            return self.dist.gather(self.tile, gather_list=parts, dst=self._dst(), group=self.group, async_op=async_op)
        self.gathered.copy_(self.tile)
        return None

    def _dst(self):
        # the global rank of the group's rank 0 (torch.distributed.gather takes a global rank)
        return self.dist.get_global_rank(self.group, 0) if self.group is not None else 0

    def step(self, seed, stream=None):
        self.render_tile(seed, stream)
        self.gather()

    def image(self) -> np.ndarray:
        """The assembled (height, width, 3) image (rank 0, after gather())."""
        if self.gathered is None:
            raise RuntimeError("the frame is gathered to rank 0 only")
        tiles = self.gathered.view(self.world_size, self.rows, self.w, 3).cpu().numpy()
        return assemble_shards(tiles, self.h, self.row_block)

    def render(self, seed):
        """The frame (rank 0) or None (the other ranks)."""
        self.step(seed)
        if self.tile_fn is None:
            self.torch.cuda.synchronize(self.device)
        return self.image() if self.rank == 0 else None

    def close(self):
        if self.scene is not None:
            self.scene.close()
            self.scene = None
