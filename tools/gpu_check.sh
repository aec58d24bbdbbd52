#!/bin/bash
# One GPU-box pass (run from the repo root under gpurun): GPU parity tests, smoke(), the default bench
# line, then the round profile (tools/profile_round.sh). Every GPU step has its own time limit and the
# chain stops at the first failure. usage: bash tools/gpu_check.sh <profile-tag> [tests|bench|prof]...
set -uo pipefail
TAG=${1:-r01}
shift || true
STEPS=${*:-tests smoke bench prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=25 -v --timeout 120 --timeout-method thread \
             > gpurun_out/gpu_tests.log 2>&1 ;;
    smoke) timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench) timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 ;;
    prof) bash tools/profile_round.sh "$TAG" > gpurun_out/prof.log 2>&1 ;;
    converge) timeout -k 10 480 python bench_converge.py --fp8 > gpurun_out/converge.json 2> gpurun_out/converge.err ;;
    convergev3) timeout -k 10 480 python bench_converge.py --preset adipose_v3 --batch 2 \
                  > gpurun_out/converge_v3.json 2> gpurun_out/converge_v3.err ;;
    proff32) bash tools/profile_round.sh "${TAG}_f32" --preset adipose_v3 --dtype f32 --size 1024 --batch 2 \
               --steps 5 --warmup 2 > gpurun_out/prof_f32.log 2>&1 ;;
    nettests) timeout -k 10 600 python -u -m pytest tests/test_gpu_network.py -x -v --timeout 120 \
             --timeout-method thread > gpurun_out/gpu_nettests.log 2>&1 ;;
    v3bench) timeout -k 10 300 python bench.py --preset adipose_v3 --batch 2 --no-cpu-baseline --no-dice \
               > gpurun_out/v3_bench_cpad64.log 2>&1 &&
             timeout -k 10 300 python bench.py --preset adipose_v3 --batch 2 --cpad 8 --no-cpu-baseline --no-dice \
               > gpurun_out/v3_bench_cpad8.log 2>&1 ;;
    v3mix) timeout -k 10 300 python bench.py --preset adipose_v3 --batch 2 --cpad 8,8,64,64 --no-cpu-baseline --no-dice \
               > gpurun_out/v3_bench_cpad_mix.log 2>&1 &&
           timeout -k 10 300 python bench_infer.py --mode tiles --steps 5 --cpad 8,8,64,64 > gpurun_out/infer_tiles_mix.log 2>&1 &&
           timeout -k 10 300 python bench_infer.py --mode tiles --steps 5 --cpad 8,64,64,64 > gpurun_out/infer_tiles_mix2.log 2>&1 ;;
    fp8) timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -v --timeout 120 --timeout-method thread \
           > gpurun_out/gpu_fp8_tests.log 2>&1 &&
         timeout -k 10 300 python bench_infer.py --mode fp8 > gpurun_out/bench_fp8.log 2>&1 ;;
    infer) timeout -k 10 300 python bench_infer.py --mode tiles --steps 5 > gpurun_out/infer_tiles.log 2>&1 &&
           timeout -k 10 300 python bench_infer.py --mode tiles --steps 5 --cpad 8 > gpurun_out/infer_tiles_cpad8.log 2>&1 &&
           timeout -k 10 400 python bench_infer.py --mode wsi > gpurun_out/infer_wsi.log 2>&1 ;;
    f32bench) timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 10 \
                --no-cpu-baseline --no-dice > gpurun_out/f32_cfg1_bench.log 2>&1 &&
              timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 \
                --warmup 2 --no-cpu-baseline --no-dice > gpurun_out/f32_1024_bench.log 2>&1 ;;
    cfg2bench) timeout -k 10 300 python bench.py --levels 4 --size 512 --batch 8 --no-cpu-baseline --no-dice \
                > gpurun_out/cfg2_bench.log 2>&1 ;;
    bnaab) timeout -k 10 300 python tools/ab_step.py --variant opt --opts "wgrad_bna_maxch=2;wgrad_bna_maxch=1" \
             > gpurun_out/bna_maxch_ab.log 2>&1 ;;
    w4) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread \
          -k "w4 or upsample_gather or tap64p_halo" > gpurun_out/w4_tests.log 2>&1 &&
        timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats,fwd --layers "L2,L3,L4" \
          --variants "fwd_w4=0;fwd_w4=1,fwd_w4_lb=0;fwd_w4=1" > gpurun_out/w4_kernels.log 2>&1 &&
        timeout -k 10 300 python tools/ab_step.py --variant opt --opts "fwd_w4=0;fwd_w4=1" > gpurun_out/w4_ab.log 2>&1 ;;
    wreg) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread \
          -k "wreg or w4 or upsample_gather or tap64p_halo" > gpurun_out/wreg_tests.log 2>&1 &&
        timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats,fwd --layers "L2,L3,L4" \
          --variants "tap64p_wreg=0;tap64p_wreg=1" > gpurun_out/wreg_kernels.log 2>&1 &&
        timeout -k 10 300 python tools/ab_step.py --variant opt --opts "tap64p_wreg=0;tap64p_wreg=1" > gpurun_out/wreg_ab.log 2>&1 ;;
    w4dbg) timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats --layers "L2,L3,L4 1024->1024" \
             --variants "fwd_w4=0;fwd_w4=1;fwd_w4_dbg=1;fwd_w4_dbg=2;fwd_w4_dbg=4;fwd_w4_dbg=7" > gpurun_out/w4_dbg.log 2>&1 ;;
    wf32) timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_network.py tests/test_engine.py \
            tests/test_gpu_configs.py -v --timeout 200 --timeout-method thread -k "f32 or wgrad or cfg1" \
            > gpurun_out/wf32_tests.log 2>&1 &&
          timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 \
            --warmup 2 --no-cpu-baseline --no-dice > gpurun_out/f32_1024_bench.log 2>&1 &&
          timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 10 \
            --no-cpu-baseline --no-dice > gpurun_out/f32_cfg1_bench.log 2>&1 ;;
    wide) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread \
          -k "tap64_persistent_matches or tap64p_halo_matches" > gpurun_out/wide_tests.log 2>&1 &&
        timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats,fwd --layers "L2,L3,L4" \
          --variants "tap64p_wide=0;tap64p_wide=1" > gpurun_out/wide_kernels.log 2>&1 &&
        timeout -k 10 300 python tools/ab_step.py --variant opt --opts "tap64p_wide=0;tap64p_wide=1" > gpurun_out/wide_ab.log 2>&1 ;;
    hwide) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread \
          -k "halop or halo_ or upsample_gather or two_chunks" > gpurun_out/hwide_tests.log 2>&1 &&
        timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats,fwd,bnr --layers "L0 64,L0 128,L1 128" \
          --variants "halop_wide=0;halop_wide=1" > gpurun_out/hwide_kernels.log 2>&1 &&
        timeout -k 10 300 python tools/ab_step.py --variant opt --opts "halop_wide=0;halop_wide=1" > gpurun_out/hwide_ab.log 2>&1 ;;
    cin8bna) timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_network.py tests/test_engine.py \
          tests/test_abi.py -v --timeout 200 --timeout-method thread -k "wgrad or unet_bn or engine or abi or cin8" \
          > gpurun_out/cin8bna_tests.log 2>&1 &&
        timeout -k 10 300 python tools/ab_step.py --variant opt --opts "wgrad_cin8_bna=0;wgrad_cin8_bna=1" > gpurun_out/cin8bna_ab.log 2>&1 ;;
    cin8w) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread \
          -k "cin8" > gpurun_out/cin8w_tests.log 2>&1 &&
        timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats --layers "L0 in8" \
          --variants "cin8_wide=0;cin8_wide=1" > gpurun_out/cin8w_kernels.log 2>&1 ;;
    hpipe) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread \
          -k "halop or halo_ or two_chunks" > gpurun_out/hpipe_tests.log 2>&1 &&
        timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats,fwd --layers "L0 64" \
          --variants "halop_wide=1;halop_wide=2" > gpurun_out/hpipe_kernels.log 2>&1 &&
        timeout -k 10 300 python tools/ab_step.py --variant opt --opts "halop_wide=1;halop_wide=2" > gpurun_out/hpipe_ab.log 2>&1 ;;
    barab) timeout -k 10 300 python tools/bench_kernels.py --kinds fwd --layers "L2 256,L3 512->512,L4 1024->1024" \
          --variants "fwd_debug=0;fwd_debug=512;fwd_debug=32;fwd_debug=544;fwd_debug=16;fwd_debug=560" > gpurun_out/barab_kernels.log 2>&1 ;;
    kpipe) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread \
          -k "kpipe or tap64p_halo or tap64_persistent or tap64_matches or f32" > gpurun_out/kpipe_tests.log 2>&1 &&
        timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats,fwd --layers "L2 256,L3 512->512,L4 1024->1024,L1 256" \
          --variants "tap64p_kpipe=0;tap64p_kpipe=1" > gpurun_out/kpipe_kernels.log 2>&1 &&
        timeout -k 10 300 python tools/bench_kernels.py --kinds bnr --layers "L2 256,L3 512->512,L4 1024->1024" \
          --variants "tap64_kpipe=0;tap64_kpipe=1" > gpurun_out/kpipe_bnr_kernels.log 2>&1 &&
        timeout -k 10 300 python tools/ab_step.py --variant opt --opts "tap64p_kpipe=0,tap64_kpipe=0;tap64p_kpipe=1,tap64_kpipe=1" > gpurun_out/kpipe_ab.log 2>&1 ;;
    bnrcfg) timeout -k 10 300 python tools/bench_kernels.py --kinds bnr --layers "L2 256,L3 512->512,L4 1024->1024,L3 1024->512,L1 256" \
          --variants "tap64p_cfg=0;tap64p_cfg=2;tap64_kpipe=1;tap64p_cfg=1,tap64p_bnr=2" > gpurun_out/bnrcfg_kernels.log 2>&1 ;;
    f8wide) timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -v --timeout 120 --timeout-method thread \
          > gpurun_out/f8wide_tests.log 2>&1 &&
        for i in 1 2; do
          timeout -k 10 300 python bench_infer.py --mode fp8 --opt tap64p_wide_f8=0 > gpurun_out/f8wide_off_$i.log 2>&1 &&
          timeout -k 10 300 python bench_infer.py --mode fp8 --opt tap64p_wide_f8=1 > gpurun_out/f8wide_on_$i.log 2>&1 || exit 1
        done ;;
    quick) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread \
             -k "wide_store or f32_lds or f32_halo or claim or halop or wgrad_persistent or tap64p" > gpurun_out/quick_tests.log 2>&1 ;;
    native) timeout -k 10 400 python -u -m pytest tests/test_gpu_native_size.py -x -v -s --timeout 200 \
              --timeout-method thread > gpurun_out/native_tests.log 2>&1 ;;
    claimab) timeout -k 10 300 python tools/ab_step.py --variant opt --opts "tap64p_claim=0;tap64p_claim=1,halop_claim=1,wgrad_halop_claim=1" \
               > gpurun_out/claim_ab.log 2>&1 ;;
    claimk) timeout -k 10 400 python tools/bench_kernels.py --kinds fwd,fwd_stats,bnr,wgrad \
              --layers "L0 64->64,L0 128->64,L1 128->128,L2 256->256,L3 512->512,L4 1024->1024" \
              --variants "tap64p_claim=0,halop_claim=0,wgrad_halop_claim=0;tap64p_claim=1,halop_claim=1,wgrad_halop_claim=1" \
              > gpurun_out/claim_kernels.log 2>&1 ;;
    claimchunk) timeout -k 10 400 python tools/bench_kernels.py --kinds fwd,wgrad \
              --layers "L0 64->64,L0 128->64,L1 128->128,L2 256->256" \
              --variants "halop_claim=0,wgrad_halop_claim=0;halop_claim=1,wgrad_halop_claim=1,halop_claim_chunk=1,wgrad_halop_claim_chunk=1;halop_claim=1,wgrad_halop_claim=1;halop_claim=1,wgrad_halop_claim=1,halop_claim_chunk=16,wgrad_halop_claim_chunk=16;halop_claim=1,wgrad_halop_claim=1,halop_claim_chunk=64,wgrad_halop_claim_chunk=64" \
              > gpurun_out/claim_chunk.log 2>&1 ;;
    probe0) timeout -k 10 400 python -u tools/contention_probe.py --blocks 0,8,32 > gpurun_out/contention_static.log 2>&1 ;;
    claimprobe) timeout -k 10 400 python -u tools/contention_probe.py --blocks 0,8,32 --opt tap64p_claim=1 --opt halop_claim=1 \
               --opt wgrad_halop_claim=1 > gpurun_out/contention_claim.log 2>&1 ;;
    contention) timeout -k 10 400 python -u tools/contention_probe.py > gpurun_out/contention.log 2>&1 ;;
    pipe2) timeout -k 10 300 python tools/bench_kernels.py --kinds fwd_stats,fwd --layers "L0 128,L1 128" \
          --variants "halop_pipe=1;halop_pipe=2;halop_pipe=2,halop_wide=2" > gpurun_out/pipe2_kernels.log 2>&1 ;;
    contention2) timeout -k 10 400 python -u tools/contention_probe.py --blocks 0,8,32 \
          --opt tap64_persist_grid=1000000 --opt halo_persist_grid=1000000 > gpurun_out/contention_nonpersist.log 2>&1 ;;
    dp2) timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
           --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline --no-dice \
           > gpurun_out/bench_dp2_gloo.log 2>&1 ;;
    dp2after) timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
           --master-port 29518 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline --no-dice --allreduce after \
           > gpurun_out/bench_dp2_gloo_after.log 2>&1 ;;
    dptests) timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -v --timeout 200 --timeout-method thread \
           > gpurun_out/dp_tests.log 2>&1 ;;
    diag) timeout -k 10 300 python -u tools/diag_bn_determinism.py > gpurun_out/diag_bn.log 2>&1 &&
          timeout -k 10 300 python -u tools/diag_f32_freeze.py > gpurun_out/diag_freeze.log 2>&1 ;;
    pmcdom) bash tools/pmc_dom.sh > gpurun_out/pmc_dom.log 2>&1 ;;
    abref) bash tools/ab_libs.sh "$(ls ab/libadipose_*.so | head -n 1)" adipose_tissue-unet_amd/libadipose_hip.so 3 \
             bench.py --no-cpu-baseline --no-dice --steps 10 > gpurun_out/ab_ref.log 2>&1 ;;
    claimk3) timeout -k 10 500 python tools/bench_kernels.py --kinds fwd,fwd_stats,bnr,wgrad \
              --layers "L0 64->64,L0 128->64,L1 128->128,L2 256->256,L3 512->512,L4 1024->1024" \
              --variants "tap64p_claim=0,halop_claim=0,wgrad_halop_claim=0;tap64p_claim=1,halop_claim=1,wgrad_halop_claim=1;tap64p_claim=1,halop_claim=1,wgrad_halop_claim=1,claim_full=1" \
              > gpurun_out/claim_kernels3.log 2>&1 ;;
    probefull) timeout -k 10 400 python -u tools/contention_probe.py --blocks 0,8,32 --opt tap64p_claim=1 --opt halop_claim=1 \
               --opt wgrad_halop_claim=1 --opt claim_full=1 > gpurun_out/contention_full.log 2>&1 ;;
    gates) timeout -k 10 600 python -u -m pytest -s -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py \
             tests/test_gpu_network.py -k "slice_vs_oracle or fallback_paths" > gpurun_out/gates.log 2>&1 ;;
    ctests) timeout -k 10 600 python -u -m pytest -s -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py \
              tests/test_gpu_configs.py tests/test_gpu_network.py \
              -k "claim or fallback_paths or slice_vs_oracle or deterministic" > gpurun_out/ctests.log 2>&1 ;;
    bprobe) timeout -k 10 500 python -u tools/contention_probe.py --buckets --blocks 8,32 > gpurun_out/bucket_probe.log 2>&1 ;;
    bprobefull) timeout -k 10 500 python -u tools/contention_probe.py --buckets --blocks 8,32 --opt claim_full=1 \
              > gpurun_out/bucket_probe_full.log 2>&1 ;;
    wtests) timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py \
              -k "tap64p_halo_matches or tap64_persistent_matches" > gpurun_out/wtests.log 2>&1 ;;
    wlines) timeout -k 10 400 python tools/bench_kernels.py --kinds fwd,fwd_stats --layers "L2 256->256,L3 512->512,L4 1024->1024" \
              --variants "tap64p_wide=1;tap64p_wide=2" > gpurun_out/wlines_kernels.log 2>&1 ;;
    wlinespmc) bash tools/pmc_dom.sh "L2 256->256,L3 512->512,L4 1024->1024" fwd,fwd_stats "tap64p_wide=2" \
              > gpurun_out/pmc_dom.log 2>&1 ;;
    wab) timeout -k 10 300 python tools/ab_step.py --variant opt --opts "tap64p_wide=1;tap64p_wide=2" > gpurun_out/wlines_ab.log 2>&1 ;;
    f8l0) timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -v --timeout 200 --timeout-method thread \
            > gpurun_out/f8l0_tests.log 2>&1 &&
          timeout -k 10 300 python bench_infer.py --mode fp8 > gpurun_out/bench_fp8_l0.log 2>&1 &&
          timeout -k 10 300 python bench_infer.py --mode fp8 --fp8-level0 0 > gpurun_out/bench_fp8_l0off.log 2>&1 ;;
    f8q) timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -v --timeout 200 --timeout-method thread \
            > gpurun_out/f8q_tests.log 2>&1 &&
          timeout -k 10 300 python bench_infer.py --mode fp8 > gpurun_out/bench_fp8_q.log 2>&1 &&
          timeout -k 10 300 python bench_infer.py --mode fp8 --opt tap64p_f8_lines=0 > gpurun_out/bench_fp8_q0.log 2>&1 ;;
    f8pipe) timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -v --timeout 200 --timeout-method thread \
              -k "halo64 or line_stores" > gpurun_out/f8pipe_tests.log 2>&1 &&
            timeout -k 10 300 python bench_infer.py --mode fp8 --opt halop_f8_pipe=0 > gpurun_out/bench_fp8_pipe0.log 2>&1 &&
            timeout -k 10 300 python bench_infer.py --mode fp8 > gpurun_out/bench_fp8_pipe1.log 2>&1 ;;
    epic) ADP_TEST_OPTS=tap64p_epic=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -v --timeout 200 --timeout-method thread \
              -k "tap64p_halo_matches or tap64_persistent_matches" > gpurun_out/epic_tests.log 2>&1 &&
          timeout -k 10 400 python tools/bench_kernels.py --kinds fwd,fwd_stats --layers "L2 256->256,L3 512->512,L4 1024->1024" \
              --variants "tap64p_epic=0;tap64p_epic=1" > gpurun_out/epic_kernels.log 2>&1 &&
          timeout -k 10 300 python tools/ab_step.py --variant opt --opts "tap64p_epic=0;tap64p_epic=1" > gpurun_out/epic_ab.log 2>&1 ;;
    f8ab) timeout -k 10 300 python bench_infer.py --mode fp8 --opt halop_f8_pipe=0 > gpurun_out/bench_fp8_pipe0.log 2>&1 &&
          timeout -k 10 300 python bench_infer.py --mode fp8 --opt tap64p_f8_lines=0 > gpurun_out/bench_fp8_q0.log 2>&1 &&
          timeout -k 10 300 python bench_infer.py --mode fp8 > gpurun_out/bench_fp8_default.log 2>&1 ;;
    f32map) timeout -k 10 300 python tools/launch_map.py --preset adipose_v3 --dtype f32 > gpurun_out/f32_map.log 2>&1 &&
            mkdir -p gpurun_out/f32kt && timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/f32kt -o kt -- \
              python3 bench.py --no-cpu-baseline --no-dice --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 3 --warmup 2 \
              > gpurun_out/f32kt/kt.log 2>&1 &&
            python3 tools/step_timeline.py gpurun_out/f32kt/kt_kernel_trace.csv > gpurun_out/f32_timeline.txt 2>&1 ;;
    f32skip) ADP_TEST_OPTS=f32_skip=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -v --timeout 200 --timeout-method thread \
              -k "f32_column_skip or tap64p_f32_halo or f32_tap_kernel" > gpurun_out/f32skip_tests.log 2>&1 &&
            timeout -k 10 400 python tools/ab_step.py --preset adipose_v3 --dtype f32 --variant opt --steps 4 \
              --opts "f32_skip=0;f32_skip=1" > gpurun_out/f32skip_ab.log 2>&1 &&
            timeout -k 10 400 python tools/ab_step.py --preset adipose_v3 --dtype f32 --variant opt --steps 4 \
              --opts "f32_eff=0;f32_eff=1" > gpurun_out/f32eff_ab.log 2>&1 ;;
    f32cfg) timeout -k 10 400 python tools/ab_step.py --preset adipose_v3 --dtype f32 --variant opt --steps 4 \
              --opts "fwd_tap64=1;fwd_tap64=3" > gpurun_out/f32cfg_ab.log 2>&1 ;;
    f32combo) timeout -k 10 400 python tools/ab_step.py --preset adipose_v3 --dtype f32 --variant opt --steps 4 \
              --opts "f32_skip=0;f32_skip=1" > gpurun_out/f32combo_ab.log 2>&1 ;;
    namefix) timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v --timeout 200 --timeout-method thread \
              -k "tap64p_wreg_matches_dma or upsample_gather_halo_forms" > gpurun_out/namefix_tests.log 2>&1 ;;
    f32eff2) timeout -k 10 400 python tools/ab_step.py --preset adipose_v3 --dtype f32 --variant opt --steps 4 \
              --opts "f32_eff=1;f32_eff=2" > gpurun_out/f32eff2_ab.log 2>&1 ;;
    names) timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py -v --timeout 200 \
              --timeout-method thread -k "tap64p or fp8 or f32" > gpurun_out/names_tests.log 2>&1 ;;
    kp) timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -v --timeout 200 --timeout-method thread \
              -k "tap64 and not tap64p" > gpurun_out/kp_tests.log 2>&1 &&
          bash tools/ab_libs.sh "$(ls ab/libadipose_*.so | head -n 1)" adipose_tissue-unet_amd/libadipose_hip.so 2 \
              tools/bench_kernels.py --kinds bnr --layers "L2 256->256,L3 512->512,L4 1024->1024" \
              --variants "tap64_kpipe=0;tap64_kpipe=1" > gpurun_out/kp_kernels_ab.log 2>&1 &&
          bash tools/ab_libs.sh "$(ls ab/libadipose_*.so | head -n 1)" adipose_tissue-unet_amd/libadipose_hip.so 3 \
              bench.py --no-cpu-baseline --no-dice --steps 10 > gpurun_out/kp_step_ab.log 2>&1 ;;
    engprobe) timeout -k 10 300 python -u tools/engine_repeat_probe.py --reps 6 --comm 1 > gpurun_out/engprobe_comm.log 2>&1 &&
              timeout -k 10 300 python -u tools/engine_repeat_probe.py --reps 6 --comm 0 > gpurun_out/engprobe_nocomm.log 2>&1 ;;
    dettests) timeout -k 10 600 python -u -m pytest tests/test_engine.py tests/test_gpu_network.py -v --timeout 200 \
              --timeout-method thread > gpurun_out/dettests.log 2>&1 ;;
    epic3) timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -v --timeout 200 --timeout-method thread \
              -k "tap64p" > gpurun_out/epic3_tests.log 2>&1 &&
          timeout -k 10 400 python tools/bench_kernels.py --kinds fwd,fwd_stats --layers "L1 128->128,L2 256->256,L3 512->512,L4 1024->1024" \
              --variants "tap64p_epic3=0;tap64p_epic3=1" > gpurun_out/epic3_kernels.log 2>&1 &&
          timeout -k 10 300 python tools/ab_step.py --variant opt --opts "tap64p_epic3=0;tap64p_epic3=1" > gpurun_out/epic3_ab.log 2>&1 ;;
    stat) timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py -v --timeout 200 --timeout-method thread \
              -k "tap64p or wgrad or halop" > gpurun_out/stat_tests.log 2>&1 &&
          timeout -k 10 400 python tools/bench_kernels.py --kinds wgrad --layers "L0 64->64,L0 128->64,L1 128->128" \
              --variants "wgrad_halop_static=0;wgrad_halop_static=1" > gpurun_out/stat_kernels.log 2>&1 &&
          timeout -k 10 300 python tools/ab_step.py --variant opt --opts "wgrad_halop_static=0,tap64p_epic3=0;wgrad_halop_static=1,tap64p_epic3=1" > gpurun_out/stat_ab.log 2>&1 ;;
    statw) timeout -k 10 300 python tools/ab_step.py --variant opt --rounds 5 --opts "wgrad_halop_static=0;wgrad_halop_static=1" > gpurun_out/statw_ab.log 2>&1 ;;
    finalinfer) timeout -k 10 300 python bench_infer.py --mode fp8 > gpurun_out/final_fp8.log 2>&1 &&
          timeout -k 10 300 python bench_infer.py --mode tiles --steps 5 > gpurun_out/final_infer_tiles.log 2>&1 &&
          timeout -k 10 300 python bench.py --levels 4 --size 512 --batch 8 --no-cpu-baseline --no-dice > gpurun_out/final_cfg2_bench.log 2>&1 ;;
    bnr3) timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_network.py -v --timeout 200 --timeout-method thread \
              -k "tap64p or bnr or bn_" > gpurun_out/bnr3_tests.log 2>&1 &&
          timeout -k 10 400 python tools/bench_kernels.py --kinds bnr --layers "L1 256->128,L2 256->256,L3 512->512,L4 1024->1024,L3 1024->512" \
              --variants "tap64p_bnr=1,tap64p_bnr_static=0;tap64p_bnr=1,tap64p_bnr_static=1;tap64p_bnr=2,tap64p_bnr_static=1" > gpurun_out/bnr3_kernels.log 2>&1 &&
          timeout -k 10 300 python tools/ab_step.py --variant opt --rounds 5 --opts "tap64p_bnr_static=0;tap64p_bnr_static=1" > gpurun_out/bnr3_ab.log 2>&1 ;;
    up1) timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -v --timeout 200 --timeout-method thread \
              -k "tap64" > gpurun_out/up1_tests.log 2>&1 &&
          timeout -k 10 400 python tools/bench_kernels.py --kinds bnr --layers "L2 256->256,L3 512->512,L4 1024->1024,L3 1024->512" \
              --variants "tap64_up1=0;tap64_up1=1" > gpurun_out/up1_kernels.log 2>&1 &&
          timeout -k 10 300 python tools/ab_step.py --variant opt --rounds 5 --opts "tap64_up1=0;tap64_up1=1" > gpurun_out/up1_ab.log 2>&1 ;;
    epic4) timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -v --timeout 200 --timeout-method thread \
              -k "tap64p" > gpurun_out/epic4_tests.log 2>&1 &&
          timeout -k 10 400 python tools/bench_kernels.py --kinds fwd,fwd_stats --layers "L1 128->128,L2 256->256,L3 512->512,L4 1024->1024" \
              --variants "tap64p_epic4=0;tap64p_epic4=1" > gpurun_out/epic4_kernels.log 2>&1 &&
          timeout -k 10 300 python tools/ab_step.py --variant opt --rounds 5 --opts "tap64p_epic4=0;tap64p_epic4=1" > gpurun_out/epic4_ab.log 2>&1 ;;
    stat2) timeout -k 10 400 python tools/bench_kernels.py --kinds wgrad --layers "L0 64->64" \
              --variants "wgrad_halop_static=1;wgrad_halop_static=2" > gpurun_out/stat2_kernels.log 2>&1 &&
          timeout -k 10 300 python tools/ab_step.py --variant opt --rounds 5 --opts "wgrad_halop_static=1;wgrad_halop_static=2" > gpurun_out/stat2_ab.log 2>&1 ;;
    cfg5) timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 300 --timeout-method thread \
            -k "cfg5" > gpurun_out/cfg5_tests.log 2>&1 ;;
    f32pmc) mkdir -p gpurun_out/f32pmc && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
              SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -f csv \
              -d gpurun_out/f32pmc -o sq -- python3 bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 \
              --steps 2 --warmup 1 --no-cpu-baseline --no-dice > gpurun_out/f32pmc/sq.log 2>&1 ;;
    bndet) timeout -k 10 300 python -u tools/diag_bn_grads.py > gpurun_out/diag_bn_grads.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "step $s rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
