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
chunks through the C++ driver (dsp_render_stft_sharded), which gathers every
chunk's rows to the root behind the next chunk's compute following the
library's gather schedule (``gather_plan``, dsp_shard_gather_plan), over a
communicator's transport:

  * ``RcclComm``      RCCL over xGMI, one process per GPU (the product);
  * ``loopback``      ranks as host threads of one process on one GPU (the
                      world > 1 driver exercised without a second GPU);
  * ``TorchComm``     a torch.distributed group (gloo) as the transport, for
                      the one-GPU multi-process rehearsal.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from . import _lib as L
from ._lib import check

TIME, CHANNELS = 0, 1


PIECE_RENDER, PIECE_MAG = 0, 1


class dsp_gather_piece(C.Structure):
    _fields_ = [("step", C.c_uint32), ("src", C.c_uint32), ("channel", C.c_uint32), ("what", C.c_uint32),
                ("src_off", C.c_uint64), ("dst_off", C.c_uint64), ("count", C.c_uint64)]


_GROUP = C.CFUNCTYPE(C.c_int, C.c_void_p)
_SEND = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p)
_RECV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p)
_DESTROY = C.CFUNCTYPE(None, C.c_void_p)


class dsp_comm_transport(C.Structure):
    _fields_ = [("group_start", _GROUP), ("group_end", _GROUP), ("send", _SEND), ("recv", _RECV),
                ("destroy", _DESTROY)]


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
    "dsp_shard_gather_plan": (C.c_int64, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_uint32, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint64,
                                          C.POINTER(C.c_uint64)]),
    "dsp_comm_init_loopback": (C.c_int, [C.c_uint32, C.c_int32, C.POINTER(C.c_void_p)]),
    "dsp_comm_init_transport": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int32,
                                          C.POINTER(C.c_void_p)]),
    "dsp_comm_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
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
# the gather schedule
# --------------------------------------------------------------------------

@dataclass(frozen=True)
class Piece:
    step: int
    src: int
    channel: int
    what: int       # PIECE_RENDER / PIECE_MAG
    src_off: int    # floats into the sender's local row
    dst_off: int    # floats into the root's whole-file row
    count: int


def gather_plan(L_total: int, C_total: int, world: int, B: int, N: int = 8192, H: int = 4096,
                mode: int = TIME, chunk: int = 0, ld: int = 4097):
    """(pieces, steps): the gather schedule dsp_render_stft_sharded follows
    (dsp_shard_gather_plan), every rank's chunk t moved to the root at step t."""
    lib = _lib()
    steps = C.c_uint64()
    n = lib.dsp_shard_gather_plan(L_total, C_total, world, B, N, H, mode, chunk, ld, None, 0, C.byref(steps))
    if n < 0:
        check(int(n), "dsp_shard_gather_plan")
    arr = (dsp_gather_piece * max(1, n))()
    lib.dsp_shard_gather_plan(L_total, C_total, world, B, N, H, mode, chunk, ld, arr, n, None)
    return [Piece(a.step, a.src, a.channel, a.what, a.src_off, a.dst_off, a.count) for a in arr[:n]], steps.value


# --------------------------------------------------------------------------
# communicators
# --------------------------------------------------------------------------

class _Comm:
    handle = None

    def _info(self):
        r, w = C.c_uint32(), C.c_uint32()
        check(_lib().dsp_comm_info(self.handle, C.byref(r), C.byref(w)), "dsp_comm_info")
        self.rank, self.world = r.value, w.value

    def gather(self, send, recv_rows, root: int = 0, stream=None):
        """Every rank's `send` (device, count floats) into the root's recv_rows[r]."""
        rows = L.chan_table([r.data_ptr() for r in recv_rows]) if recv_rows is not None else None
        check(_lib().dsp_comm_gather(self.handle, C.cast(C.c_void_p(send.data_ptr()), L.FP), send.numel(), rows,
                                     root, C.c_void_p(stream) if stream else None), "dsp_comm_gather")

    def close(self):
        h = getattr(self, "handle", None)
        if h:
            _lib().dsp_comm_destroy(h)
            self.handle = None

    def __del__(self):
        self.close()


class RcclComm(_Comm):
    """dsp_comm over RCCL inside libdspbench (xGMI), one process per GPU."""

    def __init__(self, uid: bytes, world: int, rank: int, device: int = -1):
        self.handle = C.c_void_p()
        buf = C.create_string_buffer(bytes(uid), 128)
        check(_lib().dsp_comm_init(buf, world, rank, device, C.byref(self.handle)), "dsp_comm_init")
        self._info()

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


class _Handle(_Comm):
    def __init__(self, handle):
        self.handle = handle
        self._info()


def loopback(world: int, device: int = -1) -> list:
    """dsp_comm_init_loopback: `world` communicators of one process, ranks as
    host threads sharing one GPU (each thread drives its own rank)."""
    arr = (C.c_void_p * world)()
    check(_lib().dsp_comm_init_loopback(world, device, arr), "dsp_comm_init_loopback")
    return [_Handle(C.c_void_p(arr[r])) for r in range(world)]


def _hip_runtime():
    """The HIP runtime already in this process (libdspbench's, which in a
    torch process is torch's own copy): by soname, never a second runtime."""
    import os
    L.lib()  # libdspbench (and its libamdhip64.so.7) loaded first
    try:
        return C.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    except OSError as e:  # loading a second runtime here would be fatal later
        raise RuntimeError("TorchComm: libamdhip64.so.7 is not loaded in this process (libdspbench links it; "
                           "is the library built against another HIP?)") from e


class TorchComm(_Comm):
    """A torch.distributed group (gloo) as a dsp_comm transport
    (dsp_comm_init_transport): the C++ driver's sends and recvs of device rows
    move through host tensors.  For the one-GPU multi-process rehearsal of the
    N > 1 path; the product's multi-GPU transport is RcclComm."""

    def __init__(self, group=None, device: int = -1):
        import torch.distributed as dist
        self.group = group
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        self._hip = _hip_runtime()
        self._hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self._hip.hipStreamSynchronize.argtypes = [C.c_void_p]
        self._depth, self._ops = 0, []

        def guard(fn):
            def run(*a):
                try:
                    return fn(*a)
                except Exception as e:  # a raising callback must not unwind through C
                    print(f"TorchComm transport: {e!r}", flush=True)
                    return L.DSP_ERR_INVALID
            return run

        def group_start(_u):
            self._depth += 1
            return 0

        def group_end(_u):
            self._depth -= 1
            return self._flush() if self._depth == 0 else 0

        def send(_u, buf, count, peer, stream):
            self._ops.append(("send", buf, count, peer, stream))
            return 0 if self._depth else self._flush()

        def recv(_u, buf, count, peer, stream):
            self._ops.append(("recv", buf, count, peer, stream))
            return 0 if self._depth else self._flush()

        self._fns = (_GROUP(guard(group_start)), _GROUP(guard(group_end)), _SEND(guard(send)),
                     _RECV(guard(recv)), _DESTROY(0))
        self._t = dsp_comm_transport(*self._fns)
        self.handle = C.c_void_p()
        check(_lib().dsp_comm_init_transport(C.byref(self._t), None, world, rank, device, C.byref(self.handle)),
              "dsp_comm_init_transport")
        self._info()

    def _flush(self):
        import torch
        import torch.distributed as dist
        ops, self._ops = self._ops, []
        works, recvs = [], []
        for kind, buf, count, peer, stream in ops:
            host = torch.empty(int(count), dtype=torch.float32)
            if kind == "send":  # the rows are final once the stream has passed them
                if self._hip.hipStreamSynchronize(stream) or self._hip.hipMemcpy(host.data_ptr(), buf, count * 4, 2):
                    return L.DSP_ERR_HIP
                works.append(dist.isend(host, dst=peer, group=self.group))
            else:
                works.append(dist.irecv(host, src=peer, group=self.group))
                recvs.append((host, buf, stream))
        for w in works:
            w.wait()
        for host, buf, stream in recvs:  # into the root's rows, ordered after its earlier work
            if self._hip.hipStreamSynchronize(stream) or self._hip.hipMemcpy(buf, host.data_ptr(), host.numel() * 4, 1):
                return L.DSP_ERR_HIP
        return 0


# --------------------------------------------------------------------------
# the per-rank driver
# --------------------------------------------------------------------------

def render_stft_sharded(x, L_total: int, C_total: int, B: int, sr: float, plugin, s: Shard,
                        out, mag, comm=None, root: int = 0, all_out=None, all_mag=None,
                        N: int = 8192, H: int = 4096, window: int = L.DSP_WIN_HANN, K: int | None = None,
                        chunk: int = 1 << 24, gather: bool = True, stream=None):
    """This rank's share of a sharded render + STFT, gathered to the root
    (dsp_render_stft_sharded).

    x:        this rank's file rows, local (x[c][0] = global sample s.start;
              time mode: owned + halo samples; channel mode: the file's rows
              of channels [s.chan0, s.chan0 + in_channels))
    out, mag: this rank's rows: [channels, >= ceil((owned + halo) / B) B] and
              [channels, >= frames, ld]
    all_out / all_mag: root only, [C_total, ceil(L / B) B] / [C_total, F, ld]
    comm:     a communicator (RcclComm, a loopback() entry, TorchComm), or None
              (no collective; at world 1 the rows are copied to all_out /
              all_mag)
    stream:   the HIP stream to compute on (default: the current torch stream)
    """
    K = K if K is not None else N // 2 + 1
    ld = mag.shape[-1]
    if gather and (comm is None or comm.rank == root) and (all_out is None or all_mag is None):
        raise ValueError("the root needs all_out and all_mag to gather into (gather=False to skip)")
    from .api import _exec, _rows
    in_ch = 0 if x is None else int(x.shape[0])
    lib = _lib()
    in_ptrs, _ = _rows(x) if in_ch else ([], None)
    out_ptrs, oref = _rows(out)
    mag_ptrs = [mag[c].data_ptr() for c in range(mag.shape[0])]
    ex = _exec(oref, stream=stream)
    ps = plugin.as_struct() if plugin is not None else None
    ex.flags |= plugin.exec_flags if plugin is not None else 0
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
