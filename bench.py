#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X offline-render + STFT path.

Metric (BASELINE.json): Msamples/s of the offline render + 8192-point FFT on
48 kHz stereo, at 1/2/4/8 GPUs, and the fraction of the HBM roofline.

One step = one pass of the hot path over one batch of synthetic input that
is already resident in HBM:

    IR_test render (B = 512, the reference's 10 ms @ 48 kHz block,
    wasapi_audio.cpp:456-457) of 1 h of 48 kHz stereo per GPU, and the
    8192-point Hann STFT (hop 4096, 4097 bins) of that render,
    = dsp_render_stft(...): ramp-table kernel + fused render/STFT kernel
      + render tail kernel.

Multi-GPU (launched by torch.distributed.run): the file is N hours long and
every rank renders its own hour (time-chunk sharding with an N - H = 4096
sample halo) -- no data-path collective, weak scaling.  At
N > 1 one more pass then runs the product's pipelined sharded driver
(dsp_render_stft_sharded) with the gather of every rank's render and spectra
to rank 0 over RCCL (xGMI), timed separately ("render_gather_ms", the
north_star's "final RCCL gather"), outside `value` (--no-gather skips it).

`--gpus N` outside a launcher starts the N ranks itself (torch.distributed.run
as a child process); under a launcher, WORLD_SIZE must equal N.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--minutes M]
                       [--no-cpu-baseline] [--no-gather]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dsp-bench_amd"))

METRIC = "Msamples/s offline render+8192-pt FFT, 48kHz stereo, 1/2/4/8 GPU; %HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector (packed) peak, same table
KERNEL = "stft8192_pk_kernel"
SR, CH, B, N_FFT, HOP = 48_000, 2, 512, 8192, 4096
K_BINS = N_FFT // 2 + 1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the fused kernel runs into the 1400 W package power cap within ~2 ms and
    # the clock controller overshoots before it settles (profiles/
    # r01_kernel_trace_headline_pk.txt): the defaults time the settled state
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--minutes", type=float, default=60.0, help="audio per GPU (default 1 h)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: skip the timed pass of the sharded driver with the RCCL gather to rank 0")
    ap.add_argument("--gather-timeout", type=float, default=240.0,
                    help="N > 1: seconds before a gather pass that has not finished is abandoned (the line is "
                         "printed with render_gather_error)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host WAV -> host spectra) pass")
    ap.add_argument("--no-companion", action="store_true",
                    help="headline: skip the input-reading companion pass (gain_test.cpp fused with the STFT)")
    ap.add_argument("--launch-events", action="store_true",
                    help="one-kernel workloads: bracket every launch with the library's HIP events inside the "
                         "timed region (costs 0.7-1%% of a step, profiles/r02_launch_events_ab.txt); default: "
                         "kernel_avg_ms = the timed region's stream events / steps")
    ap.add_argument("--fir-method", type=int, default=0, choices=[0, 1, 2],
                    help="fir1024: 0 auto (overlap-save), 1 direct form, 2 overlap-save")
    ap.add_argument("--workload", default="headline",
                    choices=["headline", "stft96k", "ch96k", "gain10min", "fir1024", "wav16", "wav24", "ir",
                             "generic", "generic_stft", "gain_stft", "wav16enc", "wav24enc", "biquad", "biquad_src",
                             "sine_src", "envelope_src"],
                    help="headline = IR_test + STFT 48 kHz (the metric); stft96k = BASELINE cfg 4 "
                         "(STFT of 1 h stereo 96 kHz from HBM); gain10min = cfg 2 render; "
                         "wav16 / wav24 = GPU decode of a 1 h stereo int16 / int24 WAV payload; "
                         "ch96k = BASELINE cfg 5: one 96 kHz channel per GPU through IR_test + STFT; "
                         "ir = compute_IR + fft_perform_and_get_magnitude latency (one 8192-pt frame per call); "
                         "generic = a reference plugin source through the generic driver (render only); "
                         "generic_stft = the same + the 8192-pt STFT (render, then the STFT, one stream); "
                         "gain_stft = gain_test render fused with the STFT (the input is read: the headline "
                         "shape with an input-dependent plugin); wav16enc / wav24enc = GPU encode of 1 h of "
                         "planar stereo into an interleaved int16 / int24 WAV payload; biquad = DSP_PLUGIN_BIQUAD "
                         "(plugins/biquad.cpp's low-pass as a block-parallel state scan, 1 h stereo); biquad_src / "
                         "sine_src = plugins/biquad.cpp / the reference's sine_test.cpp compiled unchanged, the "
                         "serial stateful chain (default 1 min of stereo); envelope_src = plugins/envelope_counter.cpp "
                         "(an envelope beside a block counter: a split State, 1 h stereo)")
    ap.add_argument("--sections", type=int, default=1, choices=[1, 2, 3, 4],
                    help="biquad: sections in the cascade (1 = plugins/biquad.cpp's low-pass; more add RBJ "
                         "peaking / high-pass sections)")
    ap.add_argument("--plugin", default=None,
                    choices=["gain_test", "IR_test", "static_gain_plugin", "balance", "fade_in", "buffer_test"],
                    help="generic / generic_stft: the reference plugin source (default gain_test / IR_test; "
                         "static_gain_plugin = test/static_gain_plugin.cpp, a State the callback only reads; "
                         "balance / fade_in = tests/plugins/*.cpp, per-channel / per-position gains: the "
                         "gain-table class; buffer_test = build/buffer_test.cpp, a State written through "
                         "arena pointers: the serial chain, use --minutes 1)")
    ap.add_argument("--ir-plugin", default="source", choices=["source", "enum"],
                    help="headline / ch96k: source = the reference's IR_test.cpp compiled unchanged for gfx950 "
                         "(dsp-bench_amd/modules/mod_IR_test.co) and dispatched through its probed block class "
                         "(the default: the plugin's own code on the measured path); enum = DSP_PLUGIN_IR_RAMP, "
                         "the library's restatement of the same callback (closed-form ramp)")
    ap.add_argument("--mag-ld", type=int, default=None,
                    help="headline / gain_stft / stft96k / generic_stft: row stride of the spectra in floats "
                         "(default K = 4097, rows packed); the K bins written per row are the same")
    ap.add_argument("--serial-state", action="store_true",
                    help="biquad_src / sine_src: the serial chain (DSP_EXEC_SERIAL_STATE, one lane) instead of "
                         "speculative segments (module.h dsp_state_spec_info)")
    ap.add_argument("--no-specialize", action="store_true",
                    help="generic / generic_stft: run the plugin's callback on every block "
                         "(DSP_EXEC_NO_SPECIALIZE) instead of its probed block class")
    return ap.parse_args()


def source_plugin(d, pname: str, C: int, B: int, sr: int, specialize: bool = True, serial_state: bool = False):
    """A reference plugin source compiled unchanged by the product's plugin
    compiler (hiprtc -> gfx950, dsp-bench_amd/modules/mod_<pname>.co, built by
    tools/make_plugin_modules.py) as a DSP_PLUGIN_GENERIC plugin with its
    default Parameters.  Returns (module, plugin, block class); the module
    must outlive every call that uses the plugin."""
    # (DSPB_MODULES_DIR: A/B builds of the driver, tools/build_lds_variants.sh)
    mdir = os.environ.get("DSPB_MODULES_DIR", os.path.join(REPO, "dsp-bench_amd", "modules"))
    with open(os.path.join(mdir, f"mod_{pname}.co"), "rb") as f:
        gmod = d.module.Module(f.read())
    gparams = gmod.default_parameters()
    gmod.initialize_state(gparams, C, float(sr))
    gplug = gmod.plugin(gparams, pname, specialize=specialize, serial_state=serial_state)
    block_class = "callback" if not specialize else gmod.block_class(gparams, C, B, float(sr))[0]
    return gmod, gplug, block_class


# plugin sources of this repository (tests/plugins/, dsp-bench_amd/plugins/), not the reference's
OWN_PLUGINS = {"balance": "tests/plugins", "fade_in": "tests/plugins", "biquad": "dsp-bench_amd/plugins",
               "envelope_counter": "dsp-bench_amd/plugins"}


def source_plugin_name(pname: str, block_class: str) -> str:
    origin = (f"this repository's {OWN_PLUGINS[pname]}/{pname}.cpp" if pname in OWN_PLUGINS
              else "the reference source")
    return (f"{pname}.cpp (DSP_PLUGIN_GENERIC, compiled unchanged from {origin}; block class "
            f"{block_class}: " + {"table": "its own callback's block, tiled, in the fused kernel",
                                  "gain": "the gain its callback gives, in the gain map",
                                  "gain_table": "the per-(channel, position) gains its callback gives, in the "
                                                "gain-table map",
                                  "callback": "the callback on every block"}[block_class] + ")")


def measure_companion(d, lib, args, x, out, mag, CH, B, sr, L, LD, soff, stream):
    """The headline's input-reading companion: gain_test.cpp compiled
    unchanged (block class GAIN) fused with the same STFT, on the headline's
    buffers; returns the line's `input_reading_companion` object."""
    import torch
    cmod, cplug, ccls = source_plugin(d, "gain_test", CH, B, sr)

    def cstep():
        d.render_stft(x, CH, B, float(sr), cplug, N=N_FFT, H=HOP, window=d.DSP_WIN_HANN,
                      K=K_BINS, ld=LD, out=out, mag=mag, sample_offset=soff)
    lib.dsp_kernel_timing(None, None, None)
    lib.dsp_kernel_timing_enable(1)
    cstep()
    torch.cuda.synchronize()
    lib.dsp_kernel_timing_enable(0)
    cm, cn, cb = C.c_double(), C.c_uint64(), C.c_uint64()
    lib.dsp_kernel_timing(C.byref(cm), C.byref(cn), C.byref(cb))
    for _ in range(max(0, args.warmup - 1)):
        cstep()
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    c0.record(stream)
    for _ in range(args.steps):
        cstep()
    c1.record(stream)
    torch.cuda.synchronize()
    cms = c0.elapsed_time(c1) / args.steps
    cbytes = cb.value / max(1, cn.value)
    companion = {
        "workload": ("gain_test.cpp compiled unchanged (block class " + ccls + ") fused with the same STFT: "
                     "the headline's shape with the input read"),
        "ms_per_step": round(cms, 4),
        "msamples_per_s": round(CH * L / (cms / 1e3) / 1e6, 1),
        "algorithmic_bytes_per_launch": int(cbytes),
        "frac_of_hbm": round(cbytes / (cms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4) if cn.value == 1 else None,
        "timing": f"region events over {args.steps} launches after {args.warmup} untimed, right after the "
                  "headline's passes",
    }
    return companion


# the instantiation each workload's dominant launch runs (stft_pk.hip /
# stft_pk_paths.hip: <SRC, KM, MapKind, POW2, WINC, PER, OPT, OCC>); a PMC
# summary counts only when it profiled this exact kernel
PK_INST = {
    "headline": "stft8192_pk_kernel<1, 0, (dspb::MapKind)3, true, true, 4, 65543, 2>",
    "ch96k": "stft8192_pk_kernel<1, 0, (dspb::MapKind)3, true, true, 4, 65543, 2>",
    "gain_stft": "stft8192_pk_kernel<1, 0, (dspb::MapKind)1, true, true, 0, 7, 2>",
    "stft96k": "stft8192_pk_kernel<0, 0, (dspb::MapKind)0, true, true, 0, 7, 2>",
    # generic_stft by block class (the gain-table plugins balance.cpp / fade_in.cpp)
    "generic_stft_gain_table": "stft8192_pk_kernel<1, 0, (dspb::MapKind)7, true, true, 0, 7, 2>",
    # the biquad kind at one section (one channel per tile)
    "biquad_1": "biquad_scan_kernel<1, false, 1>",
}


def pmc_key(wl: str, block_class, sections: int) -> str:
    """The PK_INST / profiles/r*_pmc_<key>.json key of a bench command."""
    if wl == "generic_stft":
        return f"generic_stft_{block_class}"
    if wl == "biquad":
        return f"biquad_{sections}"
    return wl


def pmc_traffic(workload: str, alg_bytes: float):
    """HBM bytes per launch of the workload's kernel instantiation from the
    newest committed PMC summary of the same bench command (rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE in separate passes, tools/pmc_summary.py --json:
    FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md), or (None, None, None).
    The summaries are of the default sizes: a run of another size (--minutes)
    gets no traffic figure rather than another launch's (within 0.9-1.5x of
    the algorithmic bytes counts as the same launch)."""
    import glob
    inst = PK_INST.get(workload)
    if inst is None:
        return None, None, None
    # the workload's own summaries first, then any other of the same
    # instantiation (ch96k runs the headline's kernel on as many frames)
    own = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_{workload}.json")), reverse=True)
    rest = sorted(set(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_*.json"))) - set(own), reverse=True)
    other = None
    for path in own + rest:
        doc = json.load(open(path))
        for name, m in doc.get("kernels", {}).items():
            # "<instantiation> [grid G]": one entry per launch size (tools/pmc_summary.py)
            if name.split(" [grid ")[0].endswith(inst) and "hbm_bytes" in m:
                t = float(m["hbm_bytes"])
                if alg_bytes and 0.9 <= t / alg_bytes <= 1.5:
                    return t, os.path.relpath(path, REPO), inst
                other = other or f"{os.path.relpath(path, REPO)} (a launch of another size: not used)"
    return None, other, inst


def rbj_section(kind: str, fc: float, q: float, gain_db: float = 0.0, sr: float = 48000.0):
    """An RBJ-cookbook biquad section (b0, b1, b2, a1, a2) / a0, float64 then
    float32: "lp" low-pass, "hp" high-pass, "peq" peaking EQ."""
    import math
    w0 = 2 * math.pi * fc / sr
    al, c = math.sin(w0) / (2 * q), math.cos(w0)
    A = 10 ** (gain_db / 40)
    b, a = {"lp": ([(1 - c) / 2, 1 - c, (1 - c) / 2], [1 + al, -2 * c, 1 - al]),
            "hp": ([(1 + c) / 2, -(1 + c), (1 + c) / 2], [1 + al, -2 * c, 1 - al]),
            "peq": ([1 + al * A, -2 * c, 1 - al * A], [1 + al / A, -2 * c, 1 - al / A])}[kind]
    return [b[0] / a[0], b[1] / a[0], b[2] / a[0], a[1] / a[0], a[2] / a[0]]


def cpu_baseline_generic(seconds_budget: float, pname: str = "gain_test", prefix: str = "libref_"):
    """The reference's own plugin source (gain_test.cpp by default), compiled
    with the JIT's flags (oracle/_ref/libref_<pname>.so; prefix "libplug_":
    one of this repository's plugins built the same way), called block by
    block by the oracle's render loop on one host core: chunks of 60 s
    stereo until the budget."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as o
    ref = o.RefPlugin(pname, CH, float(SR), prefix=prefix)
    chunk = SR * 60
    x = np.random.default_rng(1).uniform(-1, 1, (CH, chunk)).astype(np.float32)
    done = 0
    t0 = time.perf_counter()
    while True:
        o.render_offline([x[c] for c in range(CH)], CH, B, float(SR), ref.as_oracle())
        done += CH * chunk
        el = time.perf_counter() - t0
        if el >= seconds_budget:
            break
    own = prefix == "libplug_"
    return {"value": done / el / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port" if own else "reference",
            "sample": f"{done // CH / SR:.0f} s of 48 kHz stereo through "
                      f"{'plugins/' + pname + '.cpp built with the reference JIT flags (-Ofast, oracle/Makefile)' if own else 'the reference' + chr(39) + 's ' + pname + '.cpp (compiled from source, -Ofast)'}"
                      " and the oracle's render_audio loop (B = 512), 1 thread"}


def _cpu_threads():
    """Host threads the all-core CPU baseline uses: the CPUs this process may
    run on (sched_getaffinity), capped by OMP_NUM_THREADS when the
    environment sets it (the GPU box sets 16 per GPU; nproc there counts the
    whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(omp))) if omp and omp.isdigit() else aff, aff


def cpu_baseline(seconds_budget: float):
    """BASELINE.md section 2 on the GPU box's host cores, a bounded sample of
    the same workload (48 kHz stereo, chunks of 60 s):

      render  the reference's own IR_test.cpp, compiled from its source with
              the JIT's flags (oracle/_ref/libref_IR_test.so), called block by
              block by the oracle's render_audio loop (audio.cpp:13-175);
      STFT    Hann 8192 / 4096, 4097 bins: the oracle's fp32 radix-4 Stockham
              real FFT (a CPU restatement, not IPP: IPP is absent).

    Timed on 1 thread, then on all available threads (render chunks in
    parallel threads, OpenMP over STFT frames).  Falls back to the restated
    callback when oracle/_ref is not built."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as o
    from concurrent.futures import ThreadPoolExecutor
    threads, aff = _cpu_threads()
    chunk = SR * 60
    if o.ref_available():
        ref = o.RefPlugin("IR_test", CH, float(SR))
        plug, render_src = ref.as_oracle(), "the reference's IR_test.cpp (-Ofast JIT flags, oracle/_ref)"
    else:
        plug, render_src = o.restated_plugin("IR_test"), "the restated IR_test callback (oracle/_ref not built)"
    zero = np.zeros(chunk, np.float32)
    sub = chunk // threads // B * B

    def render_part(i):  # blocks [i sub, (i + 1) sub) of the chunk (IR_test keeps no state)
        n = sub if i < threads - 1 else chunk - sub * (threads - 1)
        return o.render_offline([zero[:n], zero[:n]], CH, B, float(SR), plug, L=n)

    def run(nt, budget):
        done, t0 = 0, time.perf_counter()
        with ThreadPoolExecutor(max_workers=nt) as ex:
            while True:
                if nt == 1:
                    out = o.render_offline([zero, zero], CH, B, float(SR), plug)
                else:
                    out = np.concatenate(list(ex.map(render_part, range(threads))), axis=1)
                for c in range(CH):
                    o.c_stft_mag_f32_r4(out[c], N_FFT, HOP, o.WIN_HANN, K_BINS, nthreads=nt)
                done += CH * chunk
                el = time.perf_counter() - t0
                if el >= budget:
                    return done / el / 1e6, done
    v1, d1 = run(1, seconds_budget / 2)
    vn, dn = run(threads, seconds_budget / 2) if threads > 1 else (v1, d1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"value": round(vn, 2), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "value_1_thread": round(v1, 2), "nproc": os.cpu_count(), "cpus_available": aff,
            "cores_note": (f"the job's CPU share: OMP_NUM_THREADS={omp} (the GPU box's share per GPU; "
                           f"sched_getaffinity reports the machine's {aff}, which other jobs share, so more threads "
                           "would oversubscribe this share, not add cores)" if omp else
                           "every CPU this process may run on (sched_getaffinity)"),
            "value_all_cpus_linear_bound": round(vn / threads * aff, 1) if aff > threads else None,
            "value_all_cpus_linear_bound_note": ("not measured: the measured per-thread rate x all the machine's "
                                                 "CPUs, an upper bound (1 -> N threads scaled "
                                                 f"{vn / max(v1, 1e-9):.1f}x here)") if aff > threads else None,
            "sample": f"{dn // CH / SR:.0f} s ({threads} threads) and {d1 // CH / SR:.0f} s (1 thread) of 48 kHz "
                      f"stereo: render through {render_src}, block by block; fp32 radix-4 Stockham real-FFT "
                      "STFT (oracle/oracle.c, OpenMP over frames). CPU restatement, not IPP"}


def bench_ir(args, dev, world, rank):
    """dsp_ir_analysis = compute_IR (plugin.cpp:17-58:
    impulse, IR_test callback over 2048 samples, 2 channels) + the Hamming
    window, 8192-point FFT and 8192 magnitudes of fft_perform_and_get_magnitude
    (dsp.cpp:53-66).  It runs once per parameter change, so it is a latency
    path: one step = one call, timed back to back."""
    import numpy as np
    import torch
    import dspbench as d
    ir_len, C_out = 2048, 2
    plugin = d.Plugin.ir_test(0.9, 0.002)
    for _ in range(args.warmup):
        d.ir_analysis(plugin, C_out=C_out, sr=float(SR), ir_len=ir_len, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        d.ir_analysis(plugin, C_out=C_out, sr=float(SR), ir_len=ir_len, device=dev)
    torch.cuda.synchronize()
    step_s = (time.perf_counter() - t0) / args.steps
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as o
        plug = o.restated_plugin("IR_test")
        n = 0
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < 2.0:
            bufs = np.zeros((C_out, ir_len), np.float32)
            bufs[:, 0] = 1.0
            o.callback_once(plug, bufs, float(SR))
            o.c_ir_magnitude(bufs[0], ir_len)
            n += 1
        cs = (time.perf_counter() - t1) / n
        cpu = {"value": round(C_out * ir_len / cs / 1e6, 3), "unit": "Msamples/s", "cores": 1, "kind": "port",
               "latency_us": round(cs * 1e6, 1),
               "sample": f"{n} analyses: the restated IR_test callback + oracle/oracle.c's float64 "
                         "Hamming window, 8192-point FFT and magnitudes (IPP is absent)"}
    alg = C_out * ir_len * 4 + 4 * ir_len * 4  # impulse-response write + magnitudes
    line = {
        "metric": METRIC, "value": round(C_out * ir_len / step_s / 1e6, 3), "unit": "Msamples/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "IR analysis (compute_IR + fft_perform_and_get_magnitude): IR_test, 2 ch x 2048 "
                               "samples, Hamming, 8192-pt FFT, 8192 magnitudes; one call per step",
                   "latency_us": round(step_s * 1e6, 1)},
        "roofline": {"bound": "hbm", "kernel": "ramp/impulse render + stft8192_pk (one frame)",
                     "achieved": round(alg / step_s / 1e9, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(alg / step_s / 1e9 / HBM_PEAK_GBPS, 6), "traffic": None,
                     "algorithmic_bytes_per_launch": alg,
                     "limiter": "launch and host-call latency: one 8192-point frame per call"},
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)


GATHER_TIMEOUT_RC = 3  # the process's exit status when the gather pass timed out


def start_gather_watchdog(seconds: float, rank: int, emit, exit_fn=None):
    """A gather that never completes (a peer lost, a transport hang) must not
    take the measured line with it, nor pass for a good run: after `seconds`
    the rank prints the line with the error (rank 0; `emit`) and leaves with
    GATHER_TIMEOUT_RC, so the launcher and the driver see a failed run.
    Returns the timer (cancel() it when the gather finishes)."""
    import threading
    exit_fn = exit_fn or os._exit

    def _expired():
        print(f"rank {rank}: the gather pass exceeded {seconds} s", file=sys.stderr, flush=True)
        emit(None, f"timed out after {seconds} s")
        sys.stdout.flush()
        exit_fn(GATHER_TIMEOUT_RC)
    dog = threading.Timer(seconds, _expired)
    dog.daemon = True
    dog.start()
    return dog


def rank_launch_cmd(n: int, argv: list[str]) -> list[str]:
    """`bench.py --gpus N` started outside a launcher: the N ranks come from
    torch.distributed.run in a child process (one process per GPU, rendezvous
    on 127.0.0.1 at a port the c10d store picks), with this script's own
    arguments; rank 0 prints the line on the inherited stdout."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
            "--rdzv-backend", "c10d", "--rdzv-endpoint", "127.0.0.1:0", "--local-addr", "127.0.0.1",
            os.path.abspath(__file__), *argv]


def check_world(gpus: int, env) -> tuple[str, str | None]:
    """What main() does for --gpus N in environment `env`: ("run", None) in a
    rank (or N = 1 unlaunched), ("launch", None) to start N ranks, or
    ("error", why) when a launcher's WORLD_SIZE disagrees with --gpus."""
    if gpus < 1:
        return "error", f"--gpus {gpus}: at least 1"
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return ("launch", None) if gpus > 1 else ("run", None)
    if int(ws) != gpus:
        return "error", f"WORLD_SIZE={ws} from the launcher but --gpus {gpus}"
    return "run", None


def main():
    args = parse()
    what, why = check_world(args.gpus, os.environ)
    if what == "error":
        print(f"bench.py: {why}", file=sys.stderr, flush=True)
        sys.exit(2)
    if what == "launch":
        # this process has made no GPU call: the ranks are children, and this
        # process exits with their launcher's status
        import subprocess
        sys.exit(subprocess.call(rank_launch_cmd(args.gpus, sys.argv[1:])))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0 and
    # gloo for the barrier / max-reduce (DSPB_BENCH_REHEARSAL=1); the real
    # multi-GPU run is one rank per GPU over RCCL
    rehearsal = os.environ.get("DSPB_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import dspbench as d
    if args.workload == "ir":
        bench_ir(args, dev, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return

    wl = args.workload
    sr = 96_000 if wl in ("stft96k", "ch96k") else SR
    # cfg 5 shards by channel (one 96 kHz channel per GPU), the rest by time
    CH = 1 if wl == "ch96k" else globals()["CH"]
    minutes = args.minutes if wl not in ("gain10min", "fir1024") or args.minutes != 60.0 else 10.0
    if (wl == "sine_src" or (wl == "biquad_src" and args.serial_state)) and args.minutes == 60.0:
        minutes = 1.0  # the serial chain: ~10 Msamples/s (sine_test's phase never forgets: serial)
    L = int(round(minutes * 60 * sr))
    L -= L % HOP  # whole hops per rank (HOP is a multiple of B)
    # the file is world * L samples long; rank r owns [r L, (r+1) L) and
    # reads a halo of the next rank's first N - H samples (dspbench/shard.py)
    if wl == "ch96k":  # cfg 5: a world-channel file, one channel run (here: one channel) per rank
        sh = d.shard.plan(L, world, rank, B, N_FFT, HOP, True, world, d.shard.CHANNELS)
        assert sh.channels == 1, sh
    else:
        sh = d.shard.plan(world * L, world, rank, B, N_FFT if wl in ("headline", "stft96k", "gain_stft") else HOP,
                          HOP, render=(wl in ("headline", "gain_stft")))
    assert sh.owned == L, (sh, L)
    L_in = sh.read_len
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = (torch.rand((CH, L_in), device=dev, generator=g) * 2 - 1) * 0.1  # synthetic WAV
    # the 10-minute files (230 MB per channel pair) would fit the 256 MiB
    # Infinity Cache between steps; steps rotate over NX copies so that every
    # step reads its input from HBM, as a one-pass offline render does
    NX = 4 if wl in ("gain10min", "fir1024") else 1
    xs = [x] + [x.clone() for _ in range(NX - 1)]
    rot = [0]

    def next_x():
        rot[0] = (rot[0] + 1) % NX
        return xs[rot[0]]
    nb = d.num_blocks(L_in, B)
    F = d.stft_frames(nb * B if wl in ("headline", "ch96k", "gain_stft") else L_in, N_FFT, HOP)
    out = (torch.empty((CH, nb * B), device=dev)
           if wl in ("headline", "ch96k", "gain10min", "fir1024", "generic", "generic_stft", "gain_stft", "biquad",
                     "biquad_src", "sine_src", "envelope_src") else None)
    if wl == "generic_stft":
        F = d.stft_frames(nb * B, N_FFT, HOP)
    LD = args.mag_ld or K_BINS
    assert LD >= K_BINS, "--mag-ld below K"
    assert LD == K_BINS or (world == 1 and wl != "ch96k"), "--mag-ld: single-GPU STFT workloads only"
    mag = (torch.empty((CH, max(F, 1), LD), device=dev)
           if wl in ("headline", "stft96k", "ch96k", "generic_stft", "gain_stft") else None)
    plugin = d.Plugin.ir_test(0.9, 0.002) if wl in ("headline", "ch96k") else d.Plugin.gain_test(0.2)
    block_class = None
    ir_note = None
    if (wl in ("headline", "ch96k") and args.ir_plugin == "source" and not os.path.exists(
            os.path.join(os.environ.get("DSPB_MODULES_DIR", os.path.join(REPO, "dsp-bench_amd", "modules")),
                         "mod_IR_test.co"))):
        # the module is compiled from /root/reference/build/IR_test.cpp by
        # build(); a tree built without the reference has only the enum
        ir_note = "mod_IR_test.co not built (no reference source at build time): DSP_PLUGIN_IR_RAMP"
        print(f"bench: {ir_note}", file=sys.stderr, flush=True)
    if wl in ("headline", "ch96k") and args.ir_plugin == "source" and ir_note is None:
        # the reference's IR_test.cpp (default Parameters {0.9, 0.002}, the
        # enum's values) compiled unchanged; its block class is probed once by
        # running its own callback, and the fused kernel renders that block
        hmod, plugin, block_class = source_plugin(d, "IR_test", CH, B, sr, specialize=not args.no_specialize)
    stream = torch.cuda.current_stream(dev)
    soff = sh.start

    lib0 = d.lib()
    alg_bytes = None  # set where the library's own launch timing does not apply
    alg_flops = None  # FLOP-bound workloads (fir1024)
    alg_desc = ("fused: C*F*(4H + 4K) B (render write + |X| write; IR_test reads no input); "
                "memory: C*F*(4H + 4K) B (each sample read once + |X| write)")
    plug_name = plugin.name
    if block_class is not None:
        plug_name = source_plugin_name("IR_test", block_class)
    if wl == "headline":
        def step():
            d.render_stft(x, CH, B, float(sr), plugin, N=N_FFT, H=HOP, window=d.DSP_WIN_HANN,
                          K=K_BINS, ld=LD, out=out, mag=mag, sample_offset=soff)
        workload = ("IR_test render (B=512) + 8192-pt Hann STFT, hop 4096, 4097 bins, "
                    f"{minutes:g} min of 48 kHz stereo per GPU")
        kname = f"{KERNEL}<render> (fused render + window + FFT + |X|)"
        if block_class == "table":
            kname = (f"{KERNEL}<render> (fused render + window + FFT + |X|; the render is IR_test.cpp's own "
                     "callback block, tiled)")
        elif block_class == "callback":
            kname = "dspb_render_lds (generic driver) then stft8192_pk<memory> on one stream"
    elif wl == "gain_stft":
        # the headline's shape with an input-dependent plugin: gain_test
        # (DSP_PLUGIN_GAIN) fused into the STFT wave, so every frame's hop is
        # read from HBM, rendered and written, and its spectrum written
        def step():
            d.render_stft(x, CH, B, float(sr), plugin, N=N_FFT, H=HOP, window=d.DSP_WIN_HANN,
                          K=K_BINS, ld=LD, out=out, mag=mag, sample_offset=soff)
        workload = ("gain_test render (B=512) fused with the 8192-pt Hann STFT, hop 4096, 4097 bins, "
                    f"{minutes:g} min of 48 kHz stereo per GPU")
        kname = f"{KERNEL}<render> (fused file read + gain + window + FFT + |X|)"
        alg_desc = "fused gain: C*F*(4H + 4H + 4K) B (file read + render write + |X| write)"
    elif wl == "ch96k":
        # the product's sharded driver (shard.h dsp_render_stft_sharded) for
        # this rank's channel, no collective in the timed step
        def step():
            d.shard.render_stft_sharded(x, L, world, B, float(sr), plugin, sh, out, mag, comm=None, gather=False,
                                        chunk=0, N=N_FFT, H=HOP, window=d.DSP_WIN_HANN, K=K_BINS)
        workload = ("BASELINE cfg 5: IR_test render (B=512) + 8192-pt Hann STFT of one 96 kHz channel "
                    f"({minutes:g} min) per GPU; channels sharded one per GPU")
        kname = f"{KERNEL}<render> (fused render + window + FFT + |X|)"
    elif wl == "stft96k":
        def step():
            d.stft_magnitude(x, N=N_FFT, H=HOP, window=d.DSP_WIN_HANN, K=K_BINS, ld=LD, out=mag)
        workload = f"8192-pt Hann STFT, hop 4096, 4097 bins, {minutes:g} min of 96 kHz stereo per GPU (cfg 4)"
        kname = f"{KERNEL}<memory> (window + FFT + |X|)"
    elif wl == "fir1024":
        # BASELINE configs[2] / SURVEY cfg 3b: 1024 taps = compute_IR(IR_test)[0:1024]
        ir, _ = d.ir_analysis(d.Plugin.ir_test(0.9, 0.002), C_out=1, sr=float(sr), device=dev)
        fplug = d.Plugin.fir(ir[0, :1024].cpu().numpy(), direct=(args.fir_method == 1))
        plug_name = "fir (1024 taps)"
        alg_desc = "C*L*(4 + 4) B (each input sample read once + each output sample written once)"

        def step():
            d.render_offline(next_x(), CH, B, float(sr), fplug, out=out)
        ols = args.fir_method != 1
        workload = (f"FIR render, 1024 taps = compute_IR(IR_test)[0:1024], B=512, {minutes:g} min of "
                    f"48 kHz stereo per GPU (cfg 3b), {'FFT overlap-save' if ols else 'direct form'}")
        if ols:  # HBM-bound: the library times it with read + write bytes
            kname = ("fir_pair_kernel (overlap-save, a channel pair as one complex 4096-pt frame, "
                     "3072 outputs per channel per frame)")
        else:
            kname = "fir_kernel (packed fp32 direct form)"
            alg_flops = 2.0 * 1024 * CH * nb * B
    elif wl == "gain10min":
        def step():
            d.render_offline(next_x(), CH, B, float(sr), plugin, out=out)
        workload = f"gain_test render (B=512), {minutes:g} min of 48 kHz stereo per GPU (cfg 2)"
        kname = "render_vec_kernel<Gain>"
        alg_bytes = CH * L_in * 8  # read + write
        alg_desc = "C*L*(4 + 4) B (read + write)"
    elif wl in ("generic", "generic_stft"):
        # a reference plugin source (gain_test.cpp /
        # IR_test.cpp) compiled by the product's plugin compiler (hiprtc ->
        # gfx950, dsp-bench_amd/modules/mod_*.co, built by
        # tools/make_plugin_modules.py) and run by the generic driver
        pname = args.plugin or ("gain_test" if wl == "generic" else "IR_test")
        gmod, gplug, block_class = source_plugin(d, pname, CH, B, sr, specialize=not args.no_specialize)
        plug_name = source_plugin_name(pname, block_class)
        if wl == "generic":
            def step():
                d.render_offline(x, CH, B, float(sr), gplug, out=out)
            workload = (f"{pname}.cpp via the generic plugin driver (B=512), {minutes:g} min of 48 kHz "
                        "stereo per GPU")
            serial = not gmod.facts.get("analyzed") or gmod.facts.get("writes_state")
            kname = ("dspb_render_st_c2b512 (generic driver: one chain through the State, LDS double buffer; "
                     "the IR analysis cannot bound its stores, DESIGN 4.6)" if serial else
                     "dspb_render_lds (generic driver, hiprtc module)" if block_class == "callback" else
                     "render_vec_kernel (the plugin's block class)")
            alg_desc = "C*L*(4 + 4) B (read + write)" if block_class != "table" else "C*L*4 B (write)"
        else:
            def step():
                d.render_stft(x, CH, B, float(sr), gplug, N=N_FFT, H=HOP, window=d.DSP_WIN_HANN,
                              K=K_BINS, ld=LD, out=out, mag=mag)
            workload = (f"{pname}.cpp via the generic plugin driver (B=512) + 8192-pt Hann STFT, hop 4096, "
                        f"4097 bins, {minutes:g} min of 48 kHz stereo per GPU")
            if block_class == "callback":
                kname = ("dspb_render_lds (generic driver) then stft8192_pk<memory> on one stream (one timed "
                         "region, dsp_render_stft)")
                alg_desc = ("C*L*(4 + 4) + C*F*4K B (file read + render write + |X| write; the STFT's re-read of "
                            "the render is extra traffic, not counted)")
            else:
                kname = (f"{KERNEL}<render> (fused render + window + FFT + |X|; the render is the plugin's own "
                         f"{'callback block, tiled' if block_class == 'table' else block_class.replace('_', ' ')})")
                alg_desc = ("fused: C*F*(4H + 4K) B (render write + |X| write; the plugin ignores its input)"
                            if block_class == "table" else
                            "fused gain: C*F*(4H + 4H + 4K) B (file read + render write + |X| write)")
    elif wl == "biquad":
        # north_star's biquad as the build-defined kind: plugins/biquad.cpp's
        # low-pass (initialize_state's coefficients) + optional sections
        import numpy as np
        rows = [d.Plugin.biquad_lowpass_coefficients(1000.0, 0.7071, float(sr))[0]]
        rows += [rbj_section(*a, sr=float(sr)) for a in
                 (("peq", 250.0, 1.5, 4.0), ("hp", 100.0, 0.7071, 0.0), ("peq", 1500.0, 2.0, 3.0))][:args.sections - 1]
        bplug = d.Plugin.biquad(np.array(rows, np.float32))
        plug_name = f"DSP_PLUGIN_BIQUAD, {args.sections} section(s): plugins/biquad.cpp's 1 kHz low-pass first"

        def step():
            d.render_offline(x, CH, B, float(sr), bplug, out=out)
        workload = (f"biquad cascade ({args.sections} section(s), direct form I, zero initial state) render "
                    f"(B=512), {minutes:g} min of 48 kHz stereo per GPU, block-parallel state scan")
        kname = f"biquad_scan_kernel<{args.sections}> (tile = 64 lanes x 32 samples, windowed look-back)"
        alg_desc = "C*L*(4 + 4) B (each input sample read once + each output sample written once)"
    elif wl in ("biquad_src", "sine_src", "envelope_src"):
        pname = {"biquad_src": "biquad", "sine_src": "sine_test", "envelope_src": "envelope_counter"}[wl]
        gmod, gplug, block_class = source_plugin(d, pname, CH, B, sr, serial_state=args.serial_state)
        plug_name = (f"{pname}.cpp compiled unchanged (DSP_PLUGIN_GENERIC; its callback writes its State: " +
                     ("the serial chain, one lane)" if args.serial_state else
                      "speculative segments checked bit for bit against the State chain, serial where they "
                      "differ)"))

        def step():
            d.render_offline(x, CH, B, float(sr), gplug, out=out)
        workload = f"{pname}.cpp via the generic plugin driver (B=512), {minutes:g} min of 48 kHz stereo per GPU"
        kname = ("dspb_render_st_c2b512 (generic driver: one chain through the State, LDS double buffer)"
                 if args.serial_state else
                 "dspb_seg_c2b512 + dspb_seg_check + dspb_seg_walk (speculative segments, DESIGN 4.6)"
                 if pname == "biquad" else
                 "dspb_seg_chain_ind_c2b512 + dspb_seg_c2b512 + dspb_seg_check + dspb_seg_walk (a split State: "
                 "the block counter's chain on 64 lanes, then speculative segments started from it; DESIGN 4.6)"
                 if pname == "envelope_counter" else
                 "dspb_seg_chain_c2b512 + dspb_seg_c2b512_rerun (a State learned never to forget: the State "
                 "chain on one lane, then every segment from its recorded State; DESIGN 4.6)")
        alg_desc = ("C*L*(4 + 4) B (read + write)" if pname in ("biquad", "envelope_counter") else
                    "C*L*4 B (write; the input is ignored)")
    elif wl in ("wav16enc", "wav24enc"):
        # SURVEY 8(f) row 1, the writer: planar float -> interleaved PCM
        # (interleave + convert, audio.h:123-133; round half to even, clip)
        bits = 16 if wl == "wav16enc" else 24
        epay = torch.empty((CH * L_in * bits // 8,), dtype=torch.uint8, device=dev)
        eptrs = d._lib.chan_table([x[c].data_ptr() for c in range(CH)])
        eex = d.api._exec(x)

        def step():
            d._lib.check(lib0.dsp_wav_encode(eptrs, CH, L_in, 1, bits, C.c_void_p(epay.data_ptr()),
                                             C.byref(eex)), "dsp_wav_encode")
        workload = f"planar float stereo -> WAV int{bits} payload (convert + interleave), {minutes:g} min of 48 kHz per GPU"
        kname = f"wav_encode_tile_kernel<{bits}, PCM, 2 ch>"
        alg_bytes = CH * L_in * (4 + bits // 8)
        plug_name = None
        alg_desc = f"C*L*(4 + {bits // 8}) B (planar float read + PCM payload write)"
    else:
        bits = 16 if wl == "wav16" else 24
        pay = torch.randint(0, 256, (CH * L_in * bits // 8,), dtype=torch.uint8, device=dev, generator=g)
        info = d._lib.dsp_wav_info(format=1, channels=CH, sample_rate=sr, bits_per_sample=bits,
                                   block_align=CH * bits // 8, frames=L_in, data_bytes=pay.numel(),
                                   n_data_chunks=1)
        wout = torch.empty((CH, L_in), device=dev)
        wptrs = d._lib.chan_table([wout[c].data_ptr() for c in range(CH)])
        wex = d.api._exec(wout)

        def step():
            d._lib.check(lib0.dsp_wav_decode(C.c_void_p(pay.data_ptr()), C.byref(info), 0, L_in, wptrs,
                                             C.byref(wex)), "dsp_wav_decode")
        workload = f"WAV int{bits} stereo payload -> planar float (decode + deinterleave), {minutes:g} min of 48 kHz per GPU"
        kname = f"wav_decode_kernel<{bits}, PCM, 2 ch>"
        alg_bytes = CH * L_in * (bits // 8 + 4)
        plug_name = None
        alg_desc = f"C*L*({bits // 8} + 4) B (PCM payload read + planar float write)"

    # the first call is cold (code objects load, the output's first touch,
    # the clock leaves idle): what an offline user rendering one file sees
    torch.cuda.synchronize()
    # one kernel per step: the timed region's own stream events give its
    # average launch duration, and no per-launch events sit between launches
    # the one-launch STFT workloads are timed by the region's stream events
    # (no events between their launches); the first call confirms one timed
    # launch per call and gives its algorithmic bytes.  The short launches
    # (fir1024, gain10min: 0.08-0.12 ms) keep events around every launch,
    # which measure the kernel alone, as rocprofv3 does (fir1024: 0.1182 ms
    # against rocprofv3's 0.1161 over all 350 launches of the same run,
    # profiles/r03_final_fir_*), not the few us between launches that the
    # region's events would add (profiles/r03_bench_all_region.jsonl)
    region_wl = (wl in ("headline", "ch96k", "gain_stft", "stft96k", "generic_stft") and
                 block_class != "callback")
    probe_launches = not args.launch_events
    launches_per_call = None
    region_timed = False
    bytes_probe = 0
    if probe_launches:
        d.lib().dsp_kernel_timing(None, None, None)
        d.lib().dsp_kernel_timing_enable(1)
    tf = time.perf_counter()
    step()
    torch.cuda.synchronize()
    first_call_ms = (time.perf_counter() - tf) * 1e3
    if probe_launches:
        d.lib().dsp_kernel_timing_enable(0)
        pm, pn, pb = C.c_double(), C.c_uint64(), C.c_uint64()
        d.lib().dsp_kernel_timing(C.byref(pm), C.byref(pn), C.byref(pb))
        region_timed = region_wl and pn.value == 1
        launches_per_call = int(pn.value)
        bytes_probe = pb.value / max(1, pn.value)
    for _ in range(max(0, args.warmup - 1)):
        step()
    torch.cuda.synchronize()

    lib = d.lib()
    lib.dsp_kernel_timing(None, None, None)  # clear
    lib.dsp_kernel_timing_enable(0 if region_timed else 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    lib.dsp_kernel_timing_enable(0)
    k_ms, k_n, k_bytes = C.c_double(), C.c_uint64(), C.c_uint64()
    lib.dsp_kernel_timing(C.byref(k_ms), C.byref(k_n), C.byref(k_bytes))
    ev_ms = ev0.elapsed_time(ev1)

    # the per-step distribution (median, p10 / p90), from a
    # separate pass with an event after every step -- those events cost a few
    # us per step, so they stay out of the timed region above
    nd = min(args.steps, 50)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(nd + 1)]
    evs[0].record(stream)
    for i in range(nd):
        step()
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    per_step = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(nd))
    pct = lambda q: per_step[min(len(per_step) - 1, int(q * (len(per_step) - 1) + 0.5))]

    step_s = max(wall, ev_ms / 1e3) / args.steps
    t = torch.tensor([step_s], dtype=torch.float64, device="cpu" if rehearsal else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    step_s = float(t.item())

    samples_per_rank = CH * L  # owned samples (the halo is re-rendered, not counted)
    value = samples_per_rank * world / step_s / 1e6

    kernel_avg_ms = k_ms.value / max(1, k_n.value)
    bytes_per_launch = k_bytes.value / max(1, k_n.value)
    if region_timed:
        kernel_avg_ms = ev_ms / args.steps
        bytes_per_launch = bytes_probe
    if k_n.value == 0 and alg_bytes is not None:  # one kernel per step, timed by the step events
        kernel_avg_ms = ev_ms / args.steps
        bytes_per_launch = alg_bytes
    achieved = bytes_per_launch / (kernel_avg_ms / 1e3) / 1e9 if kernel_avg_ms > 0 else 0.0

    # N > 1: one more pass through the product's pipelined sharded driver
    # with the gather to rank 0 (RCCL over xGMI inside libdspbench; the
    # one-GPU rehearsal uses gloo as the transport), timed on its own,
    # outside `value`
    gather_ms = None
    gather_err = None
    gather_pending = not args.no_gather and world > 1 and wl in ("headline", "ch96k")

    # the same fused kernel with a plugin that reads its input: gain_test.cpp
    # compiled unchanged (block class GAIN), the headline's shape and buffers,
    # each frame's hop read from HBM -- IR_test ignores its input, so every
    # headline frame is the same spectrum; this companion is not.  Timed as the
    # headline (region events, --warmup untimed then --steps); never `value`
    companion = None
    mdir = os.environ.get("DSPB_MODULES_DIR", os.path.join(REPO, "dsp-bench_amd", "modules"))
    if (wl == "headline" and world == 1 and not args.no_companion and
            os.path.exists(os.path.join(mdir, "mod_gain_test.co"))):
        try:
            companion = measure_companion(d, lib, args, x, out, mag, CH, B, sr, L, LD, soff, stream)
        except Exception as e:  # reported in the line; `value` stands on its own
            companion = {"error": f"{type(e).__name__}: {e}"}

    # end to end: the same hour as a 16-bit PCM WAV payload in
    # pinned host memory -> chunked H2D -> GPU decode -> render + STFT -> D2H
    # of the render and the spectra into pinned host rows
    # (dsp_render_stft_wav); never `value`
    e2e = None
    if wl == "headline" and world == 1 and not args.no_e2e:
        from dspbench import wav as dwav
        frames = L_in
        pay = torch.randint(-32768, 32768, (CH * frames,), dtype=torch.int16).view(torch.uint8).pin_memory()
        info = d._lib.dsp_wav_info(format=1, channels=CH, sample_rate=sr, bits_per_sample=16, block_align=CH * 2,
                                   frames=frames, data_bytes=pay.numel(), n_data_chunks=1)
        h_out = torch.empty((CH, nb * B), pin_memory=True)
        h_mag = torch.empty((CH, F, K_BINS), pin_memory=True)
        ts = []
        for i in range(3):  # the first call pays the slots' allocation
            torch.cuda.synchronize()
            te = time.perf_counter()
            dwav.render_stft_wav(pay, info, CH, B, float(sr), plugin, out=h_out, mag=h_mag, chunk=1 << 23,
                                 stream=stream.cuda_stream)
            ts.append((time.perf_counter() - te) * 1e3)
        e2e_ms = min(ts[1:])
        pcie = (pay.numel() + (h_out.numel() + h_mag.numel()) * 4) / (e2e_ms / 1e3) / 1e9
        e2e = {"end_to_end_ms": round(e2e_ms, 3), "first_call_ms": round(ts[0], 3),
               "msamples_per_s": round(CH * L / (e2e_ms / 1e3) / 1e6, 1),
               "host_link_gb_s": round(pcie, 1),
               "path": "16-bit stereo WAV payload in pinned host memory -> dsp_render_stft_wav (8 Mi-sample "
                       "chunks: H2D, GPU decode, fused IR_test render + STFT, D2H of render + 4097-bin spectra "
                       "into pinned host rows on an SDMA engine), best of 2 after a first call",
            "d2h_bound_ms": round((h_out.numel() + h_mag.numel()) * 4 / 57e9 * 1e3, 1),
            "d2h_bound": "the downloads alone at the 57 GB/s one SDMA engine moves device -> host "
                         "(profiles/r03_d2h_probe.txt)"}
        del pay, h_out, h_mag

    traffic, traffic_src, traffic_inst = pmc_traffic(pmc_key(wl, block_class, args.sections), bytes_per_launch)
    # the last timed render of a State-writing source plugin (module.h dsp_state_spec_info)
    state_segments = gmod.state_spec() if wl in ("biquad_src", "sine_src", "envelope_src") else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and wl == "headline":
        cpu = cpu_baseline(args.cpu_seconds)
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and wl == "generic" and args.plugin != "IR_test":
        cpu = cpu_baseline_generic(min(args.cpu_seconds, 5.0), args.plugin or "gain_test")
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and wl in ("biquad", "biquad_src"):
        cpu = cpu_baseline_generic(min(args.cpu_seconds, 8.0), "biquad", prefix="libplug_")
        if wl == "biquad" and args.sections > 1:
            cpu["note"] = "one section (plugins/biquad.cpp); the kind above runs more"
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and wl == "sine_src":
        cpu = cpu_baseline_generic(min(args.cpu_seconds, 8.0), "sine_test")
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and wl == "envelope_src":
        cpu = cpu_baseline_generic(min(args.cpu_seconds, 8.0), "envelope_counter", prefix="libplug_")

    def emit(gather_ms, gather_err):
        if rank != 0:
            return
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (uniform noise WAV in HBM; IR_test output is input-independent)"
                     if wl in ("headline", "ch96k") or (wl == "generic_stft" and "IR_test" in plug_name) else
                     f"synthetic (uniform noise in HBM; {NX} input copies used in rotation, past the Infinity Cache)"
                     if NX > 1 else "synthetic (uniform noise in HBM)"),
            "config": {
                "workload": workload,
                "plugin": plug_name,
                "block_class": block_class,
                "state_segments": state_segments,
                "mag_row_stride": LD if mag is not None else None,
                "timed_launches_per_call": launches_per_call,
                "ir_plugin": (None if wl not in ("headline", "ch96k") else
                              ir_note or ("source" if args.ir_plugin == "source" else "enum")),
                "samples_per_gpu": samples_per_rank,
                "frames_per_gpu": CH * F if mag is not None else 0,
                "sharding": ("one 96 kHz channel per GPU (a world-channel file, dsp_shard_plan CHANNELS, "
                             "dsp_render_stft_sharded), no data-path collective" if wl == "ch96k" else
                             "one independent file per GPU (a stateful plugin's state crosses time chunks: it "
                             "shards by channel or by file, never by time), no data-path collective"
                             if wl in ("biquad", "biquad_src", "sine_src", "envelope_src") else
                             "time-chunk per GPU, 4096-sample halo, no data-path collective"),
                "render_gather_ms": None if gather_ms is None else round(gather_ms, 3),
                "render_gather_error": gather_err,
                "render_gather": ("one pass of the product's pipelined sharded driver with the gather of every "
                                  "rank's render and spectra to rank 0 (dsp_render_stft_sharded over "
                                  + ("gloo, the one-GPU rehearsal)" if rehearsal else "RCCL / xGMI)")
                                  if gather_ms is not None else None),
                "first_call_ms": round(first_call_ms, 4),
                "end_to_end": e2e,
                "input_reading_companion": companion,
                "settled_step_ms_p50": round(pct(0.5), 4),
                "step_ms_p10_p50_p90": [round(pct(0.1), 4), round(pct(0.5), 4), round(pct(0.9), 4)],
                "step_ms_distribution": f"{nd} further steps, one event after each (outside the timed region)",
            },
            "roofline": ({
                "bound": "fp32-vector",
                "kernel": kname,
                "achieved": round(alg_flops / (kernel_avg_ms / 1e3) / 1e12, 2),
                "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(alg_flops / (kernel_avg_ms / 1e3) / 1e12 / FP32_PEAK_TFLOPS, 4),
                "traffic": None,
                "kernel_avg_ms": round(kernel_avg_ms, 5),
                "algorithmic": "2 * taps FLOP per output sample",
            } if alg_flops is not None else {
                "bound": "hbm",
                "kernel": kname,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": None if traffic is None else round(traffic / 1e9, 4),
                "traffic_unit": "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": traffic_src,
                "traffic_kernel": traffic_inst if traffic_src is not None else None,
                "traffic_over_algorithmic": (round(traffic / bytes_per_launch, 5)
                                             if traffic is not None and bytes_per_launch else None),
                "kernel_avg_ms": round(kernel_avg_ms, 5),
                "kernel_avg_source": ("HIP events on the launch stream around the timed region / steps (one "
                                      "kernel launch per step)" if region_timed or (k_n.value == 0 and alg_bytes)
                                      else "HIP events around every launch in the timed region (libdspbench "
                                      "dsp_kernel_timing)"),
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "algorithmic": alg_desc,
                "limiter": ("package power: the settled kernel draws the 1400 W cap at sclk ~1.8 GHz "
                            "(2.38 GHz without its stores); profiles/r01_power_ablation"
                            if wl in ("headline", "ch96k", "gain_stft") else
                            "one lane per block: the plugin callback runs serially over its block in LDS, "
                            "16 blocks per 64 KB workgroup round (DESIGN 4.6)"
                            if wl == "generic" and block_class == "callback" else
                            "the read + write stream (render_vec_kernel)" if wl == "generic" else
                            "the read + write stream and the two recurrence passes (DESIGN 4.7)" if wl == "biquad" else
                            "the serial chain: one lane runs the callback block after block (a State written "
                            "every block); DESIGN 4.6" if wl in ("biquad_src", "sine_src", "envelope_src") and
                            (args.serial_state or not (state_segments or {}).get("used")) else
                            "the State chain at its ISA floor: one lane runs the phase update frame after frame "
                            "(the callback's block arithmetic compiled away): v_add_f64 -> v_add_f64 + "
                            "v_cmp_lt_f64 -> s_nop 1 -> v_cndmask x2, measured alone at 34.3 shader cycles per "
                            "frame (14.4 ns at 2.39 GHz; a dependent v_add_f64 is 6.3, the VCC round trip the "
                            "rest: tools/diag/f64_chain_floor.hip, profiles/r06_f64_chain_floor.jsonl), then the "
                            "segments in parallel; DESIGN 4.6" if (state_segments or {}).get("chain") else
                            ("a split State: the block counter's chain on 64 lanes, then "
                             "the speculative segments as biquad_src's; DESIGN 4.6"
                             if (state_segments or {}).get("split") else
                             "segments: one lane per segment runs the callback's own chain block after block "
                            "(wave 0 of each workgroup; waves 1-3 move the blocks); the lanes are the blocks LDS "
                            "holds (18 per 76 KB workgroup, 36 per CU), so the rounds (blocks per segment + "
                            "warm-up) bound it; DESIGN 4.6")
                            if wl in ("biquad_src", "sine_src", "envelope_src") else
                            "the render (LDS-capacity-bound callbacks) then the power-capped memory STFT, "
                            "serial: DESIGN 4.6, profiles/r02_generic_stft_schedules.txt"
                            if wl == "generic_stft" and block_class == "callback" else
                            "package power, as the headline (the same fused kernel)" if wl == "generic_stft"
                            else None),
            }),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)

    if gather_pending:
        # every rank stops after --gather-timeout s, rank 0 printing the line
        # with the error, all with a non-zero status
        dog = start_gather_watchdog(args.gather_timeout, rank, emit)
        try:
            comm = d.shard.TorchComm(device=local) if rehearsal else d.shard.RcclComm.from_torch(device=local)
            Ctot = world if wl == "ch96k" else CH
            Lfile = L if wl == "ch96k" else world * L
            Lpad = d.num_blocks(Lfile, B) * B
            Ftot = d.stft_frames(Lpad, N_FFT, HOP)
            all_out = torch.empty((Ctot, Lpad), device=dev) if rank == 0 else None
            all_mag = torch.empty((Ctot, Ftot, K_BINS), device=dev) if rank == 0 else None
            torch.cuda.synchronize()
            dist.barrier()
            tg = time.perf_counter()
            d.shard.render_stft_sharded(x, Lfile, Ctot, B, float(sr), plugin, sh, out, mag, comm=comm, root=0,
                                        all_out=all_out, all_mag=all_mag, chunk=1 << 24, N=N_FFT, H=HOP,
                                        window=d.DSP_WIN_HANN, K=K_BINS)
            torch.cuda.synchronize()
            dist.barrier()
            gather_ms = (time.perf_counter() - tg) * 1e3
            comm.close()
            del all_out, all_mag
        except Exception as e:  # reported in the line; `value` stands on its own
            gather_ms, gather_err = None, f"{type(e).__name__}: {e}"
            print(f"rank {rank}: gather pass failed: {gather_err}", file=sys.stderr, flush=True)
        dog.cancel()
    emit(gather_ms, gather_err)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
