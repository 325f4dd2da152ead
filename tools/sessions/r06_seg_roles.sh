# the speculative segments' pass 1 with the work split by role (wave 0 the
# callbacks, waves 1-3 the blocks: plugin_driver_seg.inl dspb_segments_roles):
# the state-spec GPU tests, pass 1's phase clocks (tools/diag/seg_timing.py on
# modules built with DSPB_SEG_TIMING into build/seg_timing_mods), and the
# bench lines of biquad_src / envelope_src / sine_src;
# profiles/r06_seg_roles_*.  Run once per variant of the mover code.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_state_spec.py > gpurun_out/roles_state_spec.txt 2>&1 || { tail -30 gpurun_out/roles_state_spec.txt; exit 1; }
tail -1 gpurun_out/roles_state_spec.txt
timeout -k 10 300 python -u tools/diag/seg_timing.py dsp-bench_amd/build/seg_timing_mods biquad envelope_counter > gpurun_out/seg_timing_roles.jsonl 2>&1 || exit 1
for wl in biquad_src envelope_src sine_src; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline --no-e2e > gpurun_out/roles_$wl.log 2>&1 || exit 1
  tail -1 gpurun_out/roles_$wl.log | cut -c1-200
done
