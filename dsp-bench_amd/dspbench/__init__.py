"""dspbench -- MI355X-native offline render + spectrum path for DSP-Bench plugins.

All compute runs in libdspbench.so (HIP kernels for gfx950).  See DESIGN.md.
"""
from ._lib import (DSP_WIN_HAMMING, DSP_WIN_HANN, DSP_WIN_RECT, DspError, LIB_PATH,  # noqa: F401
                   lib)
from .api import (IR_BUFFER_LENGTH, Plugin, fft_forward, fft_reverse, ir_analysis,  # noqa: F401
                  minmax_decimate, num_blocks, render_loop, render_offline, render_stft, render_stft_host,
                  spectrogram_decimate,
                  stft_frames, stft_magnitude)
from . import module, shard, wav  # noqa: F401

__all__ = ["Plugin", "render_offline", "render_loop", "render_stft_host", "minmax_decimate", "spectrogram_decimate", "stft_magnitude", "render_stft", "ir_analysis",
           "fft_forward", "fft_reverse", "stft_frames", "num_blocks", "lib", "DspError",
           "DSP_WIN_HAMMING", "DSP_WIN_HANN", "DSP_WIN_RECT", "IR_BUFFER_LENGTH", "shard", "wav", "module"]
