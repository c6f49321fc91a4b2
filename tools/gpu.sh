#!/bin/bash
# GPU stages for one gpurun call:   tools/gpu.sh <stage> [<stage> ...]
# Each stage is one or more tools/gpu_step.sh steps (own time limit, log in
# gpurun_out/<name>.log); stages run in order and the call stops at the first
# fault (gpu_step.sh exits 99 on anything but pass / ordinary test failure).
#
#   smoke        __graft_entry__.smoke()
#   suite        pytest -m gpu (the whole GPU suite)
#   tests:<k>    pytest -m gpu -k <k>
#   peer8        the 8-process executor test once at the default 4 hardware
#                queues per process, per-rank LFA_TRACE / LFA_DEBUG logs under
#                gpurun_out/peer_logs, HIP runtime errors (AMD_LOG_LEVEL=1)
#   bench        driver-shaped bench (--gpus 1 --steps 20 --warmup 5) under
#                rocprofv3 --kernel-trace --stats
#   benchplain   the same without the profiler
#   pmc          the headline kernel's FETCH_SIZE / WRITE_SIZE in separate passes
#   treeput      bench.py --tune-treeput A/B (TREEPUT_VARIANTS, default 0), in
#                separate allocations and in one skewed pool
#   treetune     bench.py --tune-tree A/B (TREE_VARIANTS, default -1,12)
#   treeput_pmc  counters of the 8->8 tree_put (TREEPUT_PMC_VARIANT)
#   clat         small-collective latency: world-1 RCCL domain and 2-process
#                P2P, C-timed loop (liblfa_bench.so) and its breakdown
#   clatll       2-process P2P latency, flagged one-shot vs LL
#   solofence    direct-dispatch latency by packet fence scopes and preload
#   sizes        combine kernel durations vs size under --kernel-trace
#   host2        2-process host-buffer allreduce, default vs group chunks
#   ipc          8 processes growing P2P workspaces 4x per cycle (export path)
#   ipcab        the same with exported workspaces freed (cache 0), then kept
#   soak         random collective programs over more seeds (stress_soak.py)
#   procs        8-process one-shot latency: parent with / without a GPU context,
#                7 workers + GPU parent, 8 workers at 4 queues
#   tplayout     8->8 tree_put per buffer set and per pool pitch
#   rehearse2/4  the N > 1 bench flow at 2 / 4 ranks sharing the GPU
#   ramp         per-wave timestamps of one combine launch (ramp / drain)
#   solo         launch -> completion word of one small kernel, by part
#   tunecomb     back-to-back combine forms at 32/64/256 MiB (COMBINE_VARIANTS)
#   tablepmc     fetch / compare tables and 32 MiB buckets: kernel trace + PMC
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
S=tools/gpu_step.sh
P="rocprofv3 --kernel-trace --stats --output-format csv"
PT="python3 -u -m pytest -x -v --timeout 200 --timeout-method thread"
for stage in "$@"; do
  case "$stage" in
    smoke)
      $S smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" || exit 99 ;;
    suite)
      $S gpu_tests 1100 $PT -m gpu -q tests || exit 99 ;;
    tests:*)
      k="${stage#tests:}"
      $S "tests_$(echo "$k" | tr -c 'A-Za-z0-9_\n' '_')" 600 $PT -m gpu tests -k "$k" || exit 99 ;;
    peer8)
      mkdir -p gpurun_out/peer_logs
      PEER_LOG_DIR=gpurun_out/peer_logs LFA_TRACE=1 AMD_LOG_LEVEL=1 LFA_TEST_HW_QUEUES=4 \
        $S peer8 300 $PT -m gpu tests/test_coll_peer_gpu.py \
        -k "test_c_executor_gpu_kernels_across_processes and 8" || exit 99 ;;
    bench)
      $S prof_bench 500 $P -d gpurun_out/prof_bench -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit 99 ;;
    benchplain)
      $S bench 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit 99 ;;
    pmc)
      $S pmc_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extras && \
      $S pmc_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extras || exit 99 ;;
    treeput)
      for lay in sep skew; do
        $S "tune_treeput_$lay" 400 python3 -u bench.py --tune-treeput --treeput-layout $lay \
          --variants "${TREEPUT_VARIANTS:-0}" --tune-rounds "${TREEPUT_ROUNDS:-10}" || exit 99
      done ;;
    treetune)
      # N -> 1 tree forms over 256 MiB of inputs (TREE_VARIANTS; 12: tapered tail)
      $S tune_tree 400 python3 -u bench.py --tune-tree --variants="${TREE_VARIANTS:--1,12}" \
        --tune-rounds "${TREE_ROUNDS:-10}" || exit 99 ;;
    treeput_pmc)
      for c in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES" \
               "TA_BUSY_avr GRBM_GUI_ACTIVE" "WRITE_SIZE" "FETCH_SIZE"; do
        tag=$(echo "$c" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
        $S "treeput_pmc_$tag" 150 timeout -s KILL 140 rocprofv3 --pmc $c --output-format csv \
          -d "gpurun_out/treeput_pmc_$tag" -o run -- python3 bench.py --tune-treeput \
          --variants "${TREEPUT_PMC_VARIANT:-0}" --tune-rounds 2 || exit 99
      done ;;
    clat)
      $S clat 300 python3 -u tools/probe_latency.py || exit 99 ;;
    clatll)
      # 2-process P2P latency with the flagged one-shot (the default), then LL
      LFA_OS_LL=0 $S clat_flagged 200 python3 -u tools/probe_latency.py --skip-world1 && \
      LFA_OS_LL=1 $S clat_ll 200 python3 -u tools/probe_latency.py --skip-world1 || exit 99 ;;
    solofence)
      # direct dispatch by packet fence scopes (acquire, release) and preload
      for f in ss an aa sn; do
        LFA_DIRECT_FENCE=$f $S "solo_fence_$f" 200 python3 -u tools/probe_solo_latency.py || exit 99
      done
      LFA_DIRECT_FENCE=an LFA_DIRECT_PRELOAD=1 $S solo_fence_an_pl 200 \
        python3 -u tools/probe_solo_latency.py || exit 99 ;;
    sizes)
      $S ksizes 300 $P -d gpurun_out/ksizes -o run -- python3 bench.py --only-extra sizes || exit 99 ;;
    host2)
      $S host2 300 python3 -u tools/probe_host_group_chunk.py || exit 99 ;;
    ipc)
      $S ipc_growth 420 python3 -u tools/probe_ipc_growth.py || exit 99 ;;
    ipcab)
      # the same probe with exported workspaces freed (the old behaviour),
      # then kept (the default)
      $S ipc_growth_nocache 420 python3 -u tools/probe_ipc_growth.py --cache-bytes 0 && \
      $S ipc_growth_cache 420 python3 -u tools/probe_ipc_growth.py || exit 99 ;;
    procs)
      # one-shot latency at 8 processes: with the parent holding a GPU context
      # or not (9 or 8 processes on the GPU), 7 workers + a GPU parent, and
      # 8 workers at 4 hardware queues each
      for cfg in "8 2 -" "8 2 p" "8 1 p" "7 2 p" "8 1 -" "6 2 p" "8 3 -"; do
        set -- $cfg
        par=""; [ "$3" = p ] && par="--parent-gpu"
        $S "procs_w$1_q$2_$3" 150 python3 -u tools/probe_p2p_latency.py --world $1 --reps 100 \
          --quick --worker-queues $2 $par || exit 99
      done ;;
    soak)
      # random programs of collectives (tests/test_coll_stress.py) over more
      # seeds: device members at 2-8 processes, then a host-buffer member
      # with every 4th post refused
      $S soak_dev 560 python3 -u tools/stress_soak.py --dev --worlds 2,3,5,8 \
        --seeds "${SOAK_SEEDS:-300-309}" \
        --nops 200 && \
      $S soak_host 400 python3 -u tools/stress_soak.py --dev --worlds 2,3,5 --seeds 400-407 \
        --nops 160 --host-rank 1 --refuse-every 4 || exit 99 ;;
    ipcanchor)
      # the growth probe with a second GPU domain open across the cycles
      # (the workspace cache lives between them), then without (the cache is
      # freed at every cycle's last domain close)
      $S ipc_growth_anchor 420 python3 -u tools/probe_ipc_growth.py --anchor && \
      $S ipc_growth_noanchor 420 python3 -u tools/probe_ipc_growth.py || exit 99 ;;
    env)
      $S env 30 bash -c 'env | grep -E "^(HSA_|HIP_|GPU_|AMD_|ROC|OMP_NUM)" | sort' || exit 99 ;;
    rehearse2)
      # the N > 1 flow at 2 ranks sharing this GPU (LFA_BENCH_REHEARSE): the
      # provider rows through a peer-transfer domain, with their oracle checks
      LFA_BENCH_REHEARSE=1 $S rehearse2 600 python3 -u bench.py --gpus 2 --steps 5 \
        --warmup 2 --no-cpu || exit 99 ;;
    rehearse4)
      # the same at 4 ranks sharing this GPU (one-shots and trees at n = 4)
      LFA_BENCH_REHEARSE=1 $S rehearse4 900 python3 -u bench.py --gpus 4 --steps 5 \
        --warmup 2 --no-cpu --extras-timeout 800 || exit 99 ;;
    rehearse8)
      # the N = 8 flow with its 8 ranks and their 8 isolated extras children
      # on this one GPU (16 processes: the box's limit)
      LFA_BENCH_REHEARSE=1 $S rehearse8 1100 python3 -u bench.py --gpus 8 --steps 5 \
        --warmup 2 --no-cpu --extras-timeout 900 || exit 99 ;;
    treeputx)
      # the bench extra (fresh buffer sets rotated, median + range)
      $S treeput_extra 300 python3 -u bench.py --only-extra tree_put || exit 99 ;;
    tree5)
      # round-5 occupancy-capped forms of the N -> 1 tree against the product
      $S tune_tree5 400 python3 -u bench.py --tune-tree --variants="${TREE_VARIANTS:--1,20,21,22,23,24}" \
        --tune-rounds "${TREE_ROUNDS:-8}" || exit 99 ;;
    treeputprof)
      # the tree_put extra under rocprofv3 --kernel-trace --stats
      $S prof_treeput 300 $P -d gpurun_out/prof_treeput -o run -- python3 bench.py \
        --only-extra tree_put || exit 99 ;;
    treeput5)
      # round-5 forms against the product, 3 buffer sets rotated
      $S tune_treeput5 500 python3 -u bench.py --tune-treeput \
        --variants "${TREEPUT_VARIANTS:-0,31,32,33,34,36,37,38,35}" \
        --tune-rounds "${TREEPUT_ROUNDS:-8}" --tune-sets 3 \
        --tune-ndst "${TREEPUT_NDST:-1,8}" || exit 99 ;;
    ipctrace)
      $S ipc_growth_trace 500 python3 -u tools/probe_ipc_growth.py --trace || exit 99 ;;
    tplayout)
      $S treeput_layout 300 python3 -u tools/probe_treeput_layout.py || exit 99 ;;
    ramp)
      $S ramp 300 python3 -u tools/probe_ramp.py || exit 99 ;;
    solo)
      $S solo 200 python3 -u tools/probe_solo_latency.py || exit 99 ;;
    solopl)
      # the same with the direct-dispatch kernel's arguments preloaded
      LFA_DIRECT_PRELOAD=1 $S solo_pl 200 python3 -u tools/probe_solo_latency.py || exit 99 ;;
    tunecomb)
      $S tune_combine 500 python3 -u tools/tune_combine.py --sizes "${COMBINE_SIZES:-32,64,256}" \
        --variants "${COMBINE_VARIANTS:-30,80,81,82,83,84}" --rounds "${COMBINE_ROUNDS:-12}" || exit 99 ;;
    wsmem)
      # P2P workspace memory kinds (LFA_WS_MEM): 2-process P2P allreduce
      # latency (one-shot sizes) and bulk (two-barrier) per kind
      for kind in ${WSMEM_KINDS:-uncached coarse fine}; do
        LFA_WS_MEM=$kind $S "wsmem_$kind" 300 python3 -u tools/probe_p2p_latency.py --world 2 \
          --reps "${WSMEM_REPS:-300}" --only "p2p:${WSMEM_SIZES:-4096,65536,1048576,16777216,67108864}" || exit 99
      done ;;
    threads)
      # host-buffer combines from 4 threads: zero-copy (default), then staged
      $S threads_zc 200 python3 -u tools/probe_threads.py && \
      LFA_HOST_ZERO_COPY=0 $S threads_staged 200 python3 -u tools/probe_threads.py || exit 99 ;;
    fetchx)
      # the fetch / compare table extra (prewarmed), three times
      for i in 1 2 3; do $S "fetch_extra_$i" 200 python3 -u bench.py --only-extra fetch || exit 99; done ;;
    threads2)
      # the 2 MiB pageable case fresh and with device memory held first
      $S threads_fresh 200 python3 -u tools/probe_threads.py --sizes 2,8 --kinds pageable && \
      $S threads_hold 200 python3 -u tools/probe_threads.py --sizes 2,8 --kinds pageable --pre-alloc-gib 64 || exit 99 ;;
    fetchtune)
      FETCH_VARIANTS="${FETCH_VARIANTS:-4,6,7,8,9,10,11}" $S fetch_tune 400 python3 -u tools/probe_fetch.py --tune || exit 99 ;;
    bucketsx)
      $S buckets_extra 200 python3 -u bench.py --only-extra buckets || exit 99 ;;
    tablepmc)
      # the fetch / compare tables (256 MiB) and the 32 MiB buckets under
      # --kernel-trace --stats, then FETCH_SIZE and WRITE_SIZE in their own passes
      for x in fetch buckets; do
        $S "prof_$x" 300 $P -d "gpurun_out/prof_$x" -o run -- python3 bench.py --only-extra $x && \
        $S "pmc_${x}_fetch" 200 timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE --output-format csv \
          -d "gpurun_out/pmc_${x}_fetch" -o run -- python3 bench.py --only-extra $x && \
        $S "pmc_${x}_write" 200 timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE --output-format csv \
          -d "gpurun_out/pmc_${x}_write" -o run -- python3 bench.py --only-extra $x || exit 99
      done ;;
    *)
      echo "unknown stage $stage"; exit 2 ;;
  esac
done
