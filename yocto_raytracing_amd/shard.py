"""Frame sharding across the GPUs of one node.

Every pixel of raytrace() (src/raytrace.cpp:228-250) depends only on the read-only
scene, so a frame splits into independent row bands. Rank r of N renders the image
bands r, r+N, r+2N, ... of `band` rows each (interleaved, so that sky rows and the
dense floor rows spread evenly over the ranks); every rank renders the same padded
number of local rows (bands past the bottom of the image come back as zeros), so
the float framebuffer is gathered with ONE fixed-size all_gather (RCCL over xGMI)
and rank 0 -- or every rank -- puts the rows back in image order with one
index_select.

The band geometry is the one yrt_render implements for yrt_render_params
{band, band_stride = N, band_offset = r} (include/yrt.h): local row l of rank r is
image row ((l // band) * N + r) * band + l % band.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class BandLayout:
    height: int
    world: int
    band: int

    @property
    def nbands(self) -> int:
        return (self.height + self.band - 1) // self.band

    @property
    def bands_per_rank(self) -> int:
        return (self.nbands + self.world - 1) // self.world

    @property
    def local_rows(self) -> int:
        """rows every rank renders (padded to the largest share)"""
        return self.bands_per_rank * self.band

    def rank_rows(self, rank: int) -> np.ndarray:
        """image row of each local row of `rank`; -1 for padding rows past the image"""
        if not 0 <= rank < self.world:
            raise ValueError(f"rank {rank} outside world of {self.world}")
        l = np.arange(self.local_rows, dtype=np.int64)
        y = ((l // self.band) * self.world + rank) * self.band + l % self.band
        return np.where(y < self.height, y, -1)

    def gather_index(self) -> np.ndarray:
        """for each image row y, its row in the rank-major gathered buffer
        (rank r's local row l sits at r * local_rows + l)"""
        idx = np.empty(self.height, dtype=np.int64)
        for r in range(self.world):
            y = self.rank_rows(r)
            ok = y >= 0
            idx[y[ok]] = r * self.local_rows + np.nonzero(ok)[0]
        return idx


def render_params_band(layout: BandLayout, rank: int):
    """(band, band_stride, band_offset) and tile_h for yrt_render_params"""
    return (layout.band, layout.world, rank), layout.local_rows


def gather_frame(shard, layout: BandLayout, index, gathered=None, frame=None, group=None):
    """All-gather every rank's (local_rows, W, 4) shard and reassemble the (H, W, 4)
    frame in image order (torch tensors; any torch.distributed backend).
    `index` is torch.as_tensor(layout.gather_index()) on shard's device."""
    import torch
    import torch.distributed as dist

    if layout.world == 1:
        gathered = shard
        if frame is None and layout.local_rows == layout.height:
            return shard  # one rank renders every row in image order: the shard is the frame
    else:
        if gathered is None:
            gathered = shard.new_empty((layout.world * layout.local_rows,) + tuple(shard.shape[1:]))
        if dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(gathered, shard, group=group)
        else:  # gloo: list form
            dist.all_gather(list(gathered.chunk(layout.world)), shard, group=group)
    if frame is None:
        return torch.index_select(gathered, 0, index)
    return torch.index_select(gathered, 0, index, out=frame)
