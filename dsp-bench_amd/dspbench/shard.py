"""shard.py -- multi-GPU sharding of the render + STFT path (include/dspbench/shard.h).

SURVEY 8(e).  One process per GPU; the plan and the chunk schedule come from
libdspbench (dsp_shard_plan / dsp_shard_chunks), the same code the C++ host
and the pipelined C driver use:

  * TIME (8e(ii)): a state-free plugin (empty ``State``: gain_test, IR_test,
    no_op) renders any block independently of the blocks before it, so a long
    file splits into time chunks, one per GPU, with no data-path exchange.
    Chunk boundaries are aligned to lcm(B, H), so every rank's blocks start
    where the whole-file render's blocks start (IR_test restarts its ramp at
    each block, ref build/IR_test.cpp:40-60) and every chunk starts on a
    frame; each rank also reads (and re-renders) the first N - H samples of
    the next chunk -- the halo -- so every frame that STARTS in its chunk is
    computed locally; frame f belongs to the rank whose chunk holds f * H.
  * CHANNELS (8e(i), BASELINE configs[4]): channel-separable plugins, one
    contiguous run of channels per GPU, the whole time axis each.  Device
    channels past the file's render from zeros (audio.cpp:65-81, 138-141).

Concatenating the ranks' owned render samples and owned frames reproduces the
whole-file result exactly.  ``render_stft_sharded`` runs a rank's share in
chunks and gathers every chunk's rows to the root behind the next chunk's
compute: over RCCL inside libdspbench (``RcclComm``, dsp_render_stft_sharded),
or over a torch.distributed group (``TorchComm``: gloo on CPU, the one-GPU
rehearsal of the N > 1 path).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from . import _lib as L
from ._lib import check

TIME, CHANNELS = 0, 1


class dsp_shard(C.Structure):
    _fields_ = [("rank", C.c_uint32), ("world", C.c_uint32), ("mode", C.c_uint32), ("chan0", C.c_uint32),
                ("channels", C.c_uint32), ("start", C.c_uint64), ("owned", C.c_uint64), ("halo", C.c_uint64),
                ("frame0", C.c_uint64), ("frames", C.c_uint64)]


_SIGS = {
    "dsp_shard_plan": (C.c_int, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                 C.c_uint32, C.c_uint32, C.c_int, C.POINTER(dsp_shard)]),
    "dsp_shard_chunks": (C.c_int64, [C.POINTER(dsp_shard), C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_int, C.c_uint64, C.POINTER(dsp_shard), C.c_uint64]),
    "dsp_comm_unique_id": (C.c_int, [C.c_void_p]),
    "dsp_comm_init": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int32, C.POINTER(C.c_void_p)]),
    "dsp_comm_destroy": (None, [C.c_void_p]),
    "dsp_comm_gather": (C.c_int, [C.c_void_p, L.FP, C.c_uint64, L.FPP, C.c_uint32, C.c_void_p]),
    "dsp_render_stft_sharded": (C.c_int, [L.FPP, C.c_uint32, C.c_uint64, L.FPP, L.FPP, C.c_uint64, C.c_uint32,
                                          C.c_uint32, C.c_float, C.POINTER(L.dsp_plugin), C.c_uint32, C.c_uint32,
                                          C.c_int32, C.c_uint32, C.POINTER(dsp_shard), C.c_uint64, C.c_void_p,
                                          C.c_uint32, L.FPP, L.FPP, C.POINTER(L.dsp_exec)]),
}
_bound = False


def _lib():
    global _bound
    lib = L.lib()
    if not _bound:
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _bound = True
    return lib


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    start: int      # first owned sample (global index); pass as sample_offset
    owned: int      # owned samples
    halo: int       # samples read past the owned range (<= N - H; 0 at EOF)
    frame0: int     # first owned STFT frame (global index)
    frames: int     # owned STFT frames
    mode: int = TIME
    chan0: int = 0
    channels: int = 0

    @property
    def end(self) -> int:
        return self.start + self.owned

    @property
    def read_len(self) -> int:
        """Samples of the file this rank reads: owned + halo."""
        return self.owned + self.halo

    def _c(self) -> dsp_shard:
        return dsp_shard(self.rank, self.world, self.mode, self.chan0, self.channels, self.start, self.owned,
                         self.halo, self.frame0, self.frames)

    @staticmethod
    def _of(s: dsp_shard) -> "Shard":
        return Shard(s.rank, s.world, s.start, s.owned, s.halo, s.frame0, s.frames, s.mode, s.chan0, s.channels)


def stft_frames(L_: int, N: int, H: int) -> int:
    """Frames of an STFT over L samples (dspbench.h dsp_stft_frame_count)."""
    return 0 if L_ < N or H == 0 else (L_ - N) // H + 1


def plan(L_total: int, world: int, rank: int, B: int, N: int = 8192, H: int = 4096,
         render: bool = True, C_total: int = 2, mode: int = TIME) -> Shard:
    """The share of an L_total-sample, C_total-channel file that ``rank`` of
    ``world`` owns (dsp_shard_plan).  ``render``: frames are counted over the
    block-padded render (ceil(L / B) * B samples, as dsp_render_stft does);
    otherwise over the raw signal (dsp_stft_magnitude)."""
    if world < 1 or not 0 <= rank < world or B < 1 or H < 1 or N < H:
        raise ValueError("plan: bad world/rank/B/N/H")
    s = dsp_shard()
    check(_lib().dsp_shard_plan(L_total, C_total, world, rank, B, N, H, mode, int(render), C.byref(s)),
          "dsp_shard_plan")
    return Shard._of(s)


def chunks(s: Shard, L_total: int, B: int, N: int = 8192, H: int = 4096, render: bool = True,
           chunk: int = 0) -> list:
    """A shard's pipeline chunks (dsp_shard_chunks)."""
    lib = _lib()
    cs = s._c()
    n = lib.dsp_shard_chunks(C.byref(cs), L_total, B, N, H, int(render), chunk, None, 0)
    if n < 0:
        check(int(n), "dsp_shard_chunks")
    arr = (dsp_shard * max(1, n))()
    lib.dsp_shard_chunks(C.byref(cs), L_total, B, N, H, int(render), chunk, arr, n)
    return [Shard._of(arr[i]) for i in range(n)]


# --------------------------------------------------------------------------
# communicators
# --------------------------------------------------------------------------

class RcclComm:
    """dsp_comm: an RCCL communicator inside libdspbench (xGMI)."""

    def __init__(self, uid: bytes, world: int, rank: int, device: int = -1):
        self.world, self.rank = world, rank
        self.handle = C.c_void_p()
        self._destroy = _lib().dsp_comm_destroy
        buf = C.create_string_buffer(bytes(uid), 128)
        check(_lib().dsp_comm_init(buf, world, rank, device, C.byref(self.handle)), "dsp_comm_init")

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(_lib().dsp_comm_unique_id(buf), "dsp_comm_unique_id")
        return buf.raw

    @staticmethod
    def from_torch(group=None, device: int = -1) -> "RcclComm":
        """Rank 0 makes the id, torch.distributed broadcasts it."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [RcclComm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return RcclComm(obj[0], world, rank, device)

    def gather(self, send, recv_rows, root: int = 0, stream=None):
        """Every rank's `send` (device, count floats) into the root's recv_rows[r]."""
        rows = L.chan_table([r.data_ptr() for r in recv_rows]) if recv_rows is not None else None
        check(_lib().dsp_comm_gather(self.handle, C.cast(C.c_void_p(send.data_ptr()), L.FP), send.numel(), rows,
                                     root, C.c_void_p(stream) if stream else None), "dsp_comm_gather")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self._destroy(h)
            self.handle = None


class TorchComm:
    """A torch.distributed group as the gather transport (gloo: CPU tensors).
    The CPU tests and the one-GPU rehearsal of the N > 1 path use it; the
    product's multi-GPU path is RcclComm."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.group = group
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)

    def run(self, pieces, root: int):
        """pieces: (src rank, send tensor on src | None, recv view on root | None)."""
        import torch
        import torch.distributed as dist
        for src, send, dst in pieces:
            if src == root:
                if self.rank == root and send is not None and dst is not None and dst.data_ptr() != send.data_ptr():
                    dst.copy_(send)
            elif self.rank == root:
                buf = torch.empty(dst.shape, dtype=dst.dtype)
                dist.recv(buf, src=src, group=self.group)
                dst.copy_(buf)
            elif self.rank == src:
                dist.send(send.detach().to("cpu").contiguous(), dst=root, group=self.group)


# --------------------------------------------------------------------------
# the per-rank driver
# --------------------------------------------------------------------------

def render_stft_sharded(x, L_total: int, C_total: int, B: int, sr: float, plugin, s: Shard,
                        out, mag, comm=None, root: int = 0, all_out=None, all_mag=None,
                        N: int = 8192, H: int = 4096, window: int = L.DSP_WIN_HANN, K: int | None = None,
                        chunk: int = 1 << 24, compute=None, gather: bool = True):
    """This rank's share of a sharded render + STFT, gathered to the root.

    x:        this rank's file rows, local (x[c][0] = global sample s.start;
              time mode: owned + halo samples; channel mode: the file's rows
              of channels [s.chan0, s.chan0 + in_channels))
    out, mag: this rank's rows: [channels, >= ceil((owned + halo) / B) B] and
              [channels, >= frames, ld]
    all_out / all_mag: root only, [C_total, ceil(L / B) B] / [C_total, F, ld]
    comm:     RcclComm (or None with world 1): the pipelined C++ driver
              (dsp_render_stft_sharded); TorchComm: the same chunk schedule and
              gather pieces, driven from Python (compute: a function
              (chunk, x_view, out_view, mag_view, sample_offset) standing in for
              the GPU render, for the CPU tests).
    """
    import torch
    from .api import _exec, _rows
    K = K if K is not None else N // 2 + 1
    ld = mag.shape[-1] if hasattr(mag, "shape") else K
    if gather and (comm is None or comm.rank == root) and (all_out is None or all_mag is None):
        raise ValueError("the root needs all_out and all_mag to gather into (gather=False to skip)")
    in_ch = 0 if x is None else int(x.shape[0])
    if isinstance(comm, TorchComm):
        world, rank = comm.world, comm.rank
        plans = [plan(L_total, world, r, B, N, H, True, C_total, s.mode) for r in range(world)]
        assert plans[rank] == s, (plans[rank], s)
        rch = [chunks(p, L_total, B, N, H, True, chunk) for p in plans]
        Lpad = -(-L_total // B) * B
        for t in range(max(len(c) for c in rch)):
            if t < len(rch[rank]) and s.channels:
                c = rch[rank][t]
                o = c.start - s.start
                Lc = min(max(L_total - c.start, 0), c.owned + c.halo)
                xo = x[:, o:o + Lc] if in_ch else None
                nb = -(-Lc // B)
                oo = out[:, o:o + nb * B]
                mo = mag[:, c.frame0 - s.frame0:c.frame0 - s.frame0 + c.frames]
                if compute is not None:
                    compute(c, xo, oo, mo, c.start)
                else:
                    from .api import render_stft
                    Fc = stft_frames(nb * B, N, H)
                    if Fc > c.frames:
                        raise ValueError(f"chunk computes {Fc} frames, owns {c.frames}")
                    # (a chunk without frames still needs valid magnitude rows)
                    mrows = mag[:, c.frame0 - s.frame0:] if c.frames else mag
                    render_stft(xo, s.channels, B, sr, plugin, N=N, H=H, window=window, K=K, ld=ld,
                                out=oo, mag=mrows, sample_offset=c.start, L_file=Lc, ref=out)
                    if out.is_cuda:
                        torch.cuda.current_stream().synchronize()
            pieces = []
            for r in range(world):
                if t >= len(rch[r]):
                    continue
                c, pr = rch[r][t], plans[r]
                rlen = Lpad - c.start if c.start + c.owned >= L_total else c.owned
                o = c.start - pr.start
                for j in range(pr.channels):
                    gc = pr.chan0 + j
                    mine, onroot = r == rank, rank == root
                    pieces.append((r, out[j, o:o + rlen] if mine else None,
                                   all_out[gc, c.start:c.start + rlen] if onroot else None))
                    pieces.append((r, mag[j, c.frame0 - pr.frame0:c.frame0 - pr.frame0 + c.frames] if mine else None,
                                   all_mag[gc, c.frame0:c.frame0 + c.frames] if onroot else None))
            if gather:
                comm.run(pieces, root)
        return
    # RCCL / world 1: the pipelined C++ driver
    lib = _lib()
    in_ptrs, _ = _rows(x) if in_ch else ([], None)
    out_ptrs, oref = _rows(out)
    mag_ptrs = [mag[c].data_ptr() for c in range(mag.shape[0])]
    ex = _exec(oref)
    ps = plugin.as_struct() if plugin is not None else None
    cs = s._c()
    ao = am = None
    if gather and all_out is not None:
        ao = L.chan_table([all_out[c].data_ptr() for c in range(all_out.shape[0])])
        am = L.chan_table([all_mag[c].data_ptr() for c in range(all_mag.shape[0])])
    if not gather:
        comm = None  # no collective: this rank's share only
    st = lib.dsp_render_stft_sharded(L.chan_table(in_ptrs) if in_ptrs else None, in_ch, L_total,
                                     L.chan_table(out_ptrs), L.chan_table(mag_ptrs), ld, C_total, B, sr,
                                     C.byref(ps) if ps is not None else None, N, H, window, K, C.byref(cs), chunk,
                                     comm.handle if comm is not None else None, root, ao, am, C.byref(ex))
    check(st, "dsp_render_stft_sharded")
