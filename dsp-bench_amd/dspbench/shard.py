"""shard.py -- time-chunk sharding of one long render + STFT across ranks.

SURVEY §8e(ii): a state-free plugin (empty ``State``: gain_test, IR_test,
no_op) renders any block independently of the blocks before it, so a long
file splits into time chunks, one per GPU, with no data-path exchange:

  * chunk boundaries are aligned to lcm(B, H), so every rank's blocks start
    where the whole-file render's blocks start (IR_test restarts its ramp at
    each block, ref build/IR_test.cpp:40-60) and every chunk starts on a frame;
  * each rank also reads (and re-renders) the first N - H samples of the next
    chunk -- the halo -- so every frame that STARTS in its chunk is computed
    locally; halos are recomputed, never exchanged;
  * frame f belongs to the rank whose chunk holds sample f * H.

Concatenating the ranks' owned render samples and owned frames reproduces
the whole-file result exactly (tests/test_shard.py checks it on CPU with the
oracle and gloo, tests/test_gpu_parity.py on the GPU).
"""
from __future__ import annotations

import math
from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    start: int      # first owned sample (global index); pass as sample_offset
    owned: int      # owned samples
    halo: int       # samples read past the owned range (<= N - H; 0 at EOF)
    frame0: int     # first owned STFT frame (global index)
    frames: int     # owned STFT frames

    @property
    def end(self) -> int:
        return self.start + self.owned

    @property
    def read_len(self) -> int:
        """Samples of the file this rank reads: owned + halo."""
        return self.owned + self.halo


def stft_frames(L: int, N: int, H: int) -> int:
    """Frames of an STFT over L samples (dspbench.h dsp_stft_frame_count)."""
    return 0 if L < N or H == 0 else (L - N) // H + 1


def plan(L_total: int, world: int, rank: int, B: int, N: int = 8192, H: int = 4096,
         render: bool = True) -> Shard:
    """The chunk of an L_total-sample file that ``rank`` of ``world`` owns.

    ``render``: frames are counted over the block-padded render
    (ceil(L / B) * B samples, as dsp_render_stft does); otherwise over the
    raw signal (dsp_stft_magnitude)."""
    if world < 1 or not 0 <= rank < world or B < 1 or H < 1 or N < H:
        raise ValueError("plan: bad world/rank/B/N/H")
    unit = B * H // math.gcd(B, H)
    units = -(-L_total // unit)
    u0, u1 = rank * units // world, (rank + 1) * units // world
    start = min(u0 * unit, L_total)
    end = min(u1 * unit, L_total)
    last = end >= L_total
    halo = 0 if last else min(N - H, L_total - end)
    L_frames = (-(-L_total // B) * B) if render else L_total
    F_total = stft_frames(L_frames, N, H)
    f0 = min(start // H, F_total)
    f1 = F_total if last else min(-(-end // H), F_total)
    return Shard(rank, world, start, end - start, halo, f0, max(0, f1 - f0))
