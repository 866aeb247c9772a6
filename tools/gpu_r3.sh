#!/bin/bash
# GPU session script (rounds 3-4): GPU tests, smoke, default bench, optional extra
# steps selected by $STEPS (space-separated: gemmcal prof). Every GPU step has
# its own limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-r3}"
STEPS="${STEPS:-tests bench}"
for s in $STEPS; do
  case $s in
    tests)
      rm -f gpurun_out/parity_${TAG}.jsonl
      MAECLIP_PARITY_OUT=gpurun_out/parity_${TAG}.jsonl timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
      tail -3 gpurun_out/pytest_gpu_${TAG}.log ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { tail -30 gpurun_out/smoke_${TAG}.log; exit 1; }
      tail -1 gpurun_out/smoke_${TAG}.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
      cat gpurun_out/bench_${TAG}.json ;;
    benchq)
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --steps 20 > gpurun_out/benchq_${TAG}.json 2> gpurun_out/benchq_${TAG}.err || { tail -30 gpurun_out/benchq_${TAG}.err; exit 1; }
      cat gpurun_out/benchq_${TAG}.json ;;
    benchdp)   # the data-parallel code path at world 1 (RCCL group, gathers, bucketed all-reduce)
      timeout -k 10 300 python -u bench.py --dp --no-cpu-baseline --no-parity --steps 20 > gpurun_out/benchdp_${TAG}.json 2> gpurun_out/benchdp_${TAG}.err || { tail -30 gpurun_out/benchdp_${TAG}.err; exit 1; }
      cat gpurun_out/benchdp_${TAG}.json ;;
    gemmcal)
      timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gemmcal_${TAG}.jsonl 2>&1 || { tail -30 gpurun_out/gemmcal_${TAG}.jsonl; exit 1; }
      cat gpurun_out/gemmcal_${TAG}.jsonl ;;
    gemmepi)
      GEMM_SET=epi timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gemmepi_${TAG}.jsonl 2>&1 || { tail -30 gpurun_out/gemmepi_${TAG}.jsonl; exit 1; }
      cat gpurun_out/gemmepi_${TAG}.jsonl ;;
    testk)   # a -k selection of the GPU tests ($TESTK)
      MAECLIP_PARITY_OUT=gpurun_out/parity_${TAG}.jsonl timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "$TESTK" --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_k_${TAG}.log 2>&1 || { tail -40 gpurun_out/pytest_k_${TAG}.log; exit 1; }
      tail -3 gpurun_out/pytest_k_${TAG}.log ;;
    cliploss)
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/cliploss_${TAG} -o run --output-format csv -- \
        python tools/clip_loss_bench.py > gpurun_out/cliploss_${TAG}.jsonl 2> gpurun_out/cliploss_${TAG}.err || { tail -30 gpurun_out/cliploss_${TAG}.err; exit 1; }
      cat gpurun_out/cliploss_${TAG}.jsonl ;;
    hbprof)  # hipBLASLt kernel names / durations for the production shapes (calibration only)
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/hbprof_${TAG} -o run --output-format csv -- \
        python tools/gemm_bench.py > gpurun_out/hbprof_${TAG}.log 2>&1 || { tail -30 gpurun_out/hbprof_${TAG}.log; exit 1; }
      tail -3 gpurun_out/hbprof_${TAG}.log ;;
    gridscan)
      MAECLIP_LIB=$PWD/mae_clip_amd/libmaeclip_dev.so timeout -k 10 200 python -u tools/gemm_grid_scan.py > gpurun_out/gridscan_${TAG}.jsonl 2>&1 || { tail -30 gpurun_out/gridscan_${TAG}.jsonl; exit 1; }
      cat gpurun_out/gridscan_${TAG}.jsonl ;;
    abattn)
      timeout -k 10 400 bash tools/ab_attn_libs.sh mae_clip_amd/libmaeclip_base.so mae_clip_amd/libmaeclip_dev.so > gpurun_out/abattn_${TAG}.txt 2>&1 || { tail -30 gpurun_out/abattn_${TAG}.txt; exit 1; }
      cat gpurun_out/abattn_${TAG}.txt ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
        python bench.py --no-cpu-baseline --no-parity > gpurun_out/prof_${TAG}.log 2>&1 || { tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
      tail -1 gpurun_out/prof_${TAG}.log ;;
    mbo)     # micro-batch stream overlap probe (tools/mb_overlap.py)
      timeout -k 10 200 python -u tools/mb_overlap.py dec 2 > gpurun_out/mbo_${TAG}.txt 2>&1 &&
      timeout -k 10 200 python -u tools/mb_overlap.py enc 2 >> gpurun_out/mbo_${TAG}.txt 2>&1 || { tail -30 gpurun_out/mbo_${TAG}.txt; exit 1; }
      cat gpurun_out/mbo_${TAG}.txt ;;
    abnt)    # same-box whole-step A/B: pending non-temporal LN / attention stores
      timeout -k 10 600 bash tools/ab_bench.sh mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_nt.so 3 > gpurun_out/abnt_${TAG}.txt 2>&1 || { tail -30 gpurun_out/abnt_${TAG}.txt; exit 1; }
      cat gpurun_out/abnt_${TAG}.txt ;;
    sq)      # main-loop rate at large square shapes vs hipBLASLt
      GEMM_SET=sq timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/sq_${TAG}.jsonl 2>&1 || { tail -30 gpurun_out/sq_${TAG}.jsonl; exit 1; }
      cat gpurun_out/sq_${TAG}.jsonl ;;
    layout)  # KC x KC vs KC x RC, padded leading dimensions (tools/gemm_layout_probe.py)
      timeout -k 10 300 python -u tools/gemm_layout_probe.py > gpurun_out/layout_${TAG}.jsonl 2>&1 || { tail -30 gpurun_out/layout_${TAG}.jsonl; exit 1; }
      cat gpurun_out/layout_${TAG}.jsonl ;;
    v6)      # GEMM v6 vs v4: bitwise equality + time (tools/gemm6_probe.py)
      timeout -k 10 500 python -u tools/gemm6_probe.py > gpurun_out/v6_${TAG}.jsonl 2>&1 || { tail -40 gpurun_out/v6_${TAG}.jsonl; exit 1; }
      cat gpurun_out/v6_${TAG}.jsonl ;;
    mbscan)  # micro-batch count x hardware queues, same box (tools/mb_scan.sh)
      timeout -k 10 900 bash tools/mb_scan.sh > gpurun_out/mbscan_${TAG}.txt 2>&1 || { tail -30 gpurun_out/mbscan_${TAG}.txt; exit 1; }
      cat gpurun_out/mbscan_${TAG}.txt ;;
    v6split) # v6 main-loop streams timed apart (tools/v6_stream_split.sh)
      timeout -k 10 900 bash tools/v6_stream_split.sh > gpurun_out/v6split_${TAG}.txt 2>&1 || { tail -30 gpurun_out/v6split_${TAG}.txt; exit 1; }
      cat gpurun_out/v6split_${TAG}.txt ;;
    v6reg)   # register-staged v6 main loop (-DV6_REG build) vs v4
      MAECLIP_LIB=$PWD/mae_clip_amd/libmaeclip_v6reg.so timeout -k 10 500 python -u tools/gemm6_probe.py > gpurun_out/v6reg_${TAG}.jsonl 2>&1 || { tail -40 gpurun_out/v6reg_${TAG}.jsonl; exit 1; }
      cat gpurun_out/v6reg_${TAG}.jsonl ;;
    pmcstep) # in-step PMC traffic of the bench's dominant launch (tools/pmc_instep.sh)
      TAG=$TAG PICK=$PMC_PICK timeout -k 10 900 bash tools/pmc_instep.sh "$PMC_KN" "$PMC_GX" "$PMC_KEY" > gpurun_out/pmcstep_${TAG}.txt 2>&1 || { tail -30 gpurun_out/pmcstep_${TAG}.txt; exit 1; }
      tail -2 gpurun_out/pmcstep_${TAG}.txt ;;
    mbstack) # micro-batch count per stack width (tools/mb_stack_scan.sh)
      timeout -k 10 900 bash tools/mb_stack_scan.sh > gpurun_out/mbstack_${TAG}.txt 2>&1 || { tail -30 gpurun_out/mbstack_${TAG}.txt; exit 1; }
      cat gpurun_out/mbstack_${TAG}.txt ;;
    attnstamps) # per-phase cycle split of the attention backward (ATTN_STAMPS build)
      MAECLIP_LIB=$PWD/mae_clip_amd/libmaeclip_stamps.so timeout -k 10 200 python -u tools/attn_stamps.py 256 197 16 32 > gpurun_out/attnstamps_${TAG}.txt 2>&1 &&
      MAECLIP_LIB=$PWD/mae_clip_amd/libmaeclip_stamps.so timeout -k 10 200 python -u tools/attn_fwd_stamps.py 256 197 16 32 >> gpurun_out/attnstamps_${TAG}.txt 2>&1 || { tail -30 gpurun_out/attnstamps_${TAG}.txt; exit 1; }
      cat gpurun_out/attnstamps_${TAG}.txt ;;
    pmcattn) # SQ counters of the decoder attention forward and backward (tools/pmc_attn.sh)
      PMCDIR=gpurun_out/pmca_fwd_${TAG} timeout -k 10 500 bash tools/pmc_attn.sh 256 197 16 32 0 > gpurun_out/pmcattn_${TAG}.txt 2>&1 &&
      PMCDIR=gpurun_out/pmca_bwd_${TAG} timeout -k 10 500 bash tools/pmc_attn.sh 256 197 16 32 1 >> gpurun_out/pmcattn_${TAG}.txt 2>&1 || { tail -30 gpurun_out/pmcattn_${TAG}.txt; exit 1; }
      cat gpurun_out/pmcattn_${TAG}.txt ;;
    plainlib) # plain bf16 GEMMs on the vendor library, whole-step A/B (tools/plain_lib_ab.sh)
      timeout -k 10 900 bash tools/plain_lib_ab.sh > gpurun_out/plainlib_${TAG}.txt 2>&1 || { tail -30 gpurun_out/plainlib_${TAG}.txt; exit 1; }
      cat gpurun_out/plainlib_${TAG}.txt ;;
    plainprobe) # per-shape own vs vendor plain GEMMs (tools/plain_gemm_probe.py)
      timeout -k 10 400 python -u tools/plain_gemm_probe.py > gpurun_out/plainprobe_${TAG}.jsonl 2>&1 || { tail -30 gpurun_out/plainprobe_${TAG}.jsonl; exit 1; }
      cat gpurun_out/plainprobe_${TAG}.jsonl ;;
    ownprobe) # per-shape own (stream-K) vs own data-parallel vs vendor (tools/own_vs_vendor_probe.py)
      timeout -k 10 500 python -u tools/own_vs_vendor_probe.py > gpurun_out/ownprobe_${TAG}.jsonl 2>&1 || { tail -30 gpurun_out/ownprobe_${TAG}.jsonl; exit 1; }
      cat gpurun_out/ownprobe_${TAG}.jsonl ;;
    cfgs)    # C1 / C4 bf16 / C4 fp8 bench lines (tools/cfg_runs.sh)
      TAG=$TAG timeout -k 10 1100 bash tools/cfg_runs.sh > gpurun_out/cfgs_${TAG}.txt 2>&1 || { tail -30 gpurun_out/cfgs_${TAG}.txt; exit 1; }
      cat gpurun_out/cfgs_${TAG}.txt ;;
    fp8lib)  # C4 fp8 with / without the vendor fp8 GEMMs (tools/fp8_lib_ab.sh)
      timeout -k 10 1100 bash tools/fp8_lib_ab.sh > gpurun_out/fp8lib_${TAG}.txt 2>&1 || { tail -30 gpurun_out/fp8lib_${TAG}.txt; exit 1; }
      cat gpurun_out/fp8lib_${TAG}.txt ;;
    fp8probe) # C4 fp8 shapes own vs vendor (tools/fp8_vendor_probe.py)
      timeout -k 10 300 python -u tools/fp8_vendor_probe.py > gpurun_out/fp8probe_${TAG}.jsonl 2>&1 || { tail -30 gpurun_out/fp8probe_${TAG}.jsonl; exit 1; }
      cat gpurun_out/fp8probe_${TAG}.jsonl ;;
    asyncloss) # loss read before / after queueing the next step (tools/async_loss_ab.sh)
      timeout -k 10 900 bash tools/async_loss_ab.sh > gpurun_out/asyncloss_${TAG}.txt 2>&1 || { tail -30 gpurun_out/asyncloss_${TAG}.txt; exit 1; }
      cat gpurun_out/asyncloss_${TAG}.txt ;;
    boundary) # GPU idle time between two replays of the captured step (tools/step_boundary_ab.sh)
      timeout -k 10 1500 bash tools/step_boundary_ab.sh > gpurun_out/boundary_${TAG}.txt 2>&1 || { tail -30 gpurun_out/boundary_${TAG}.txt; exit 1; }
      grep -v "^\[" gpurun_out/boundary_${TAG}.txt ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
