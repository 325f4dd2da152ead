set -e
mkdir -p gpurun_out/r06d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -w -o /tmp/f64_chain_floor tools/diag/f64_chain_floor.hip
timeout -k 10 60 /tmp/f64_chain_floor > gpurun_out/r06d/f64_chain_floor.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for S in 1 4; do
 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex biquad_scan -d gpurun_out/r06d/pmc_s${S}_a -o run --output-format csv -- python bench.py --workload biquad --sections $S --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-companion > gpurun_out/r06d/pmc_s${S}_a.log 2>&1
 timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-include-regex biquad_scan -d gpurun_out/r06d/pmc_s${S}_b -o run --output-format csv -- python bench.py --workload biquad --sections $S --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-companion > gpurun_out/r06d/pmc_s${S}_b.log 2>&1
done
