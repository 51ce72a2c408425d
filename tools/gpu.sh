# One parameterised GPU-box script for every record in profiles/ (replaces the round-1..3
# one-off wrappers).  Each task writes gpurun_out/<tag>_*; steps are chained with && and
# each GPU step has its own time limit.
#
#   gpurun --timeout 1100 -- bash tools/gpu.sh <task>[,<task>...] [tag]
#
# tasks
#   suite     the whole GPU test suite + smoke()                            (GPUTEST-style record)
#   bench     the driver's command, default / fp32 / per-rank-8 / large-batch benches (JSON lines)
#   rehearse  N=1 and a 2-rank gloo rehearsal of the multi-rank bench flow on the one GPU (also with
#             CSED_TIME_PATHS=1), bench.py --device cpu --gpus 2/4/8 under torchrun (N concurrent
#             imports + rendezvous, bringup_s) and tools/rccl_init_probe.py (one-rank RCCL bring-up)
#   trace     rocprofv3 kernel traces: default (B=64), per-rank 8, B=1024 / 8192 fp16, fp32 64 / 8
#   stages    in-kernel stage stamps (train B=64 / 8, tile B=1024, fp32 B=64) + update stamps
#   exchange  loopback exchange table (tools/exchange_loopback.py) + step breakdown
#             (tools/exchange_trace.py) + the exchange / fault-injection / comm tests
#   tiletrace per-step breakdown (tools/exchange_trace.py) of the large-batch step: lenet_tile span,
#             gaps, lenet_update FC / CONV roles at B = 1024 and 8192
#   pmc       three rocprofv3 --pmc passes over the train kernel (B=64), one over B=8,
#             and three over the tile kernel (B=1024)
#   modular   the modular engine: fusion + op tests, graph step times (B = 64), a kernel trace
#   abops     tools/op_probe.py (per-op launch times of the modular step) for every ab/*_C.so build
#   modpmc    one rocprofv3 --pmc pass over the modular step's kernels (fetch / memory waits)
#   ddp       tools/ddp_overlap.py: the modular engine's bucketed reducer, per-bucket all-reduce on the
#             comm stream vs after backward, step times + overlap share from kernel traces
#   ab        same-box A/B of ab/A_C.so vs ab/B_C.so (tools/ab_build.sh REV) at global batch
#             64 and 8 (+ AB_ARGS), N_AB alternations (default 3)
#   abtile    same-box A/B of ab/A_C.so vs ab/B_C.so at global batch 1024 / 8192 fp16 (lenet_tile)
#   pmctile   the three PMC passes over the tile kernel only (B = 1024)
#   abenv     same-box A/B of one build under ENV_A vs ENV_B (BENCH_ARGS / AB_ARGS / N_AB)
#   abcfg     same-box A/B of ab/A_C.so vs ab/B_C.so over several bench configs (AB_CFGS, N_AB)
#   splitk    rocprofv3 kernel stats of the B = 8192 fp16 step for ab/A_C.so vs ab/B_C.so, alternating
#             (was gpu_r5j.sh), and the loopback world-8 soak
#   ipcmem    the exchange receive buffer's allocation: uncached (default) vs CSED_IPC_MEM=finegrained
#             (was gpu_ipcmem.sh)
#   bringtrace rocprofv3 HIP-API + kernel + memory-copy trace of the bench bring-up, summarised
#   wgradab   same-build A/B of the conv weight-gradient staging depth at B = 4096 (op times, step)
#   epoch0    the reference span on a fresh process, stamped: bench.py --epoch0-stamps at N = 1 (bf16,
#             fp32) + the driver's own command
TASKS=${1:?task list}
T=${2:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
py() { timeout -k 10 "$@"; }

task_suite() {
  cd $R && py 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/${T}_tests.log 2>&1
  local rc=$?
  grep -E "passed|failed" $O/${T}_tests.log | tail -1 > $O/${T}_tests_summary.txt
  [ $rc -le 1 ] && py 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 && [ $rc -eq 0 ]
}

task_bench() {
  cd $R && py 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_bench_driver.json 2>$O/${T}_bench_driver.err && \
  py 200 python bench.py > $O/${T}_bench_default.json 2>$O/${T}_bench_default.err && \
  py 200 python bench.py --dtype fp32 > $O/${T}_bench_fp32.json 2>$O/${T}_bench_fp32.err && \
  py 200 python bench.py --global-batch 8 --steps 3000 --warmup 300 --no-epoch > $O/${T}_bench_b8.json 2>$O/${T}_bench_b8.err && \
  py 200 python bench.py --global-batch 8 --loopback-world 8 --steps 3000 --warmup 300 --no-epoch > $O/${T}_bench_lb8.json 2>$O/${T}_bench_lb8.err && \
  py 200 python bench.py --global-batch 1024 --dtype fp16 --steps 300 --warmup 30 --no-epoch > $O/${T}_bench_1024.json 2>$O/${T}_bench_1024.err && \
  py 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 > $O/${T}_bench_8192.json 2>$O/${T}_bench_8192.err
}

task_rehearse() {
  cd $R && py 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_reh_n1.json 2>$O/${T}_reh_n1.err && \
  py 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 > $O/${T}_reh_gloo2.json 2>$O/${T}_reh_gloo2.err && \
  CSED_TIME_PATHS=1 py 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-fp32-record > $O/${T}_reh_gloo2_tp.json 2>$O/${T}_reh_gloo2_tp.err && \
  py 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 20 --warmup 5 > $O/${T}_reh_nccl2.json 2>$O/${T}_reh_nccl2.err && \
  for n in 2 4 8; do
    py 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --device cpu --steps 2 --warmup 1 > $O/${T}_reh_cpu$n.json 2>$O/${T}_reh_cpu$n.err || return 1
  done && \
  py 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29611 tools/rccl_init_probe.py > $O/${T}_rccl_init.log 2>&1
}

task_trace() {
  cd /tmp && export TMPDIR=/tmp && \
  py 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt64 -o run -- python3 $R/bench.py --steps 300 --warmup 30 --no-epoch --no-fp32-record > $O/${T}_kt64.log 2>&1 && \
  py 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt8 -o run -- python3 $R/bench.py --global-batch 8 --steps 300 --warmup 30 --no-epoch --no-fp32-record > $O/${T}_kt8.log 2>&1 && \
  py 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt1024 -o run -- python3 $R/bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch --no-fp32-record > $O/${T}_kt1024.log 2>&1 && \
  py 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt8192 -o run -- python3 $R/bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 --no-epoch --no-fp32-record > $O/${T}_kt8192.log 2>&1 && \
  py 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_ktf32 -o run -- python3 $R/bench.py --dtype fp32 --steps 300 --warmup 30 --no-epoch > $O/${T}_ktf32.log 2>&1
}

task_stages() {
  cd $R && py 120 python tools/stage_profile.py 64 > $O/${T}_stage64.log 2>&1 && \
  py 120 python tools/stage_profile.py 8 > $O/${T}_stage8.log 2>&1 && \
  py 120 python tools/stage_profile_tile.py 1024 > $O/${T}_stage_tile1024.log 2>&1 && \
  py 120 python tools/stage_profile_f32.py 64 > $O/${T}_stage_f32.log 2>&1 && \
  py 120 python tools/update_profile.py 8 > $O/${T}_update8.log 2>&1 && \
  py 120 python tools/update_profile.py 8192 > $O/${T}_update8192.log 2>&1
}

task_exchange() {
  cd $R && py 300 python -u tools/exchange_loopback.py 8 16 32 64 > $O/${T}_loopback.log 2>&1 && \
  py 300 python -u tools/exchange_trace.py --batch 8 16 32 64 --worlds 1 2 4 8 > $O/${T}_xtrace.log 2>&1 && \
  py 600 python -u -m pytest tests/test_exchange_loopback_gpu.py tests/test_fault_injection_gpu.py tests/test_comm_gpu.py -v --timeout 240 --timeout-method thread > $O/${T}_xtests.log 2>&1
}

task_tiletrace() {
  cd $R && py 300 python -u tools/exchange_trace.py --batch 1024 8192 --worlds 1 --steps 16 > $O/${T}_tiletrace.log 2>&1
}

task_modular() {  # the modular (per-op) engine: fusion / op tests, graph step times at B = 64, a kernel trace
  cd $R && py 600 python -u -m pytest tests/test_modular_fusion_gpu.py tests/test_kernels_gpu.py tests/test_modular_graph_gpu.py \
    tests/test_dropout_pin_gpu.py tests/test_fused_gpu.py tests/test_kernels_f32_gpu.py tests/test_engine_gpu.py \
    -x -v --timeout 200 --timeout-method thread > $O/${T}_modtests.log 2>&1 && \
  py 200 python -u tools/ddp_overlap.py --graph graph --steps 500 > $O/${T}_modddp.log 2>&1 && \
  py 200 python -u tools/ddp_overlap.py --graph graph --steps 500 --loader >> $O/${T}_modddp.log 2>&1 && \
  cd /tmp && export TMPDIR=/tmp && \
  py 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_modkt -o run -- python3 $R/tools/ddp_overlap.py --trace --batch 64 --mode nocomm --bucket-mb 25 --graph graph > $O/${T}_modkt.log 2>&1 && \
  cd $R && python3 tools/ddp_overlap.py --phases $(ls $O/${T}_modkt/*kernel_trace.csv $O/${T}_modkt/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/${T}_modkt_phases.json 2>&1 && \
  cd /tmp && py 300 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_modkt4096 -o run -- python3 $R/tools/ddp_overlap.py --trace --batch 4096 --mode nocomm --bucket-mb 25 --graph graph > $O/${T}_modkt4096.log 2>&1 && \
  cd $R && python3 tools/ddp_overlap.py --phases $(ls $O/${T}_modkt4096/*kernel_trace.csv $O/${T}_modkt4096/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/${T}_modkt4096_phases.json 2>&1
}

task_modpmc() {  # two PMC passes over the modular step's kernels: waits / fetch, then the MFMA share
  cd /tmp && export TMPDIR=/tmp && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/${T}_modpmc -o run -- python3 $R/tools/ddp_overlap.py --trace --batch ${MOD_B:-64} --mode nocomm --bucket-mb 25 --graph eager > $O/${T}_modpmc.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU --output-format csv -d $O/${T}_modpmc2 -o run -- python3 $R/tools/ddp_overlap.py --trace --batch ${MOD_B:-64} --mode nocomm --bucket-mb 25 --graph eager > $O/${T}_modpmc2.log 2>&1 && \
  cd $R && python3 tools/kernel_counters.py --summarize $(ls $O/${T}_modpmc/*counter_collection.csv $O/${T}_modpmc/*/*counter_collection.csv 2>/dev/null | head -1) $(ls $O/${T}_modpmc2/*counter_collection.csv $O/${T}_modpmc2/*/*counter_collection.csv 2>/dev/null | head -1) > $O/${T}_modpmc_summary.log 2>&1
}

task_abops() {  # per-op launch times of the modular step (tools/op_probe.py) for every ab/*_C.so build
  cd $R && rm -f $O/${T}_abops.log && \
  for i in $(seq ${N_AB:-2}); do for so in ab/*_C.so; do
    echo "== $so" >> $O/${T}_abops.log && \
    CSED_NATIVE_SO=$R/$so py 120 python tools/op_probe.py >> $O/${T}_abops.log 2>&1 || return 1
  done; done
}

task_ddp() {  # the modular engine's bucketed reducer: step times per mode + overlap from kernel traces
  cd $R && py 200 python -u tools/ddp_overlap.py > $O/${T}_ddp.log 2>&1 && \
  py 300 python -u tools/ddp_overlap.py --batch 4096 --steps 50 >> $O/${T}_ddp.log 2>&1 && \
  cd /tmp && export TMPDIR=/tmp && \
  for m in overlap serial; do
    py 200 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_ddp_$m -o run -- python3 $R/tools/ddp_overlap.py --trace --batch 4096 --mode $m --bucket-mb 0.01 > $O/${T}_ddp_$m.log 2>&1 && \
    python3 $R/tools/ddp_overlap.py --parse $O/${T}_ddp_$m/run_kernel_trace.csv >> $O/${T}_ddp.log 2>&1 || return 1
  done
}

pmc3() {  # pmc3 <tag> <kernel_counters.py args>
  local t=$1; shift
  cd /tmp && export TMPDIR=/tmp && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d $O/${t}1 -o run -- python3 $R/tools/kernel_counters.py "$@" > $O/${t}1.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $O/${t}2 -o run -- python3 $R/tools/kernel_counters.py "$@" > $O/${t}2.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM --output-format csv -d $O/${t}3 -o run -- python3 $R/tools/kernel_counters.py "$@" > $O/${t}3.log 2>&1 && \
  cd $R && python3 tools/kernel_counters.py --summarize $O/${t}1/run_counter_collection.csv $O/${t}2/run_counter_collection.csv $O/${t}3/run_counter_collection.csv > $O/${t}_summary.log 2>&1
}

task_pmc() {
  pmc3 ${T}_pmc64 64 200 && pmc3 ${T}_pmc8 8 200 && pmc3 ${T}_pmc1024 1024 100
}

task_ab() {
  cd $R && rm -f $O/${T}_ab.log && \
  for i in $(seq ${N_AB:-3}); do for b in 64 8; do for v in A B; do
    echo "$v B=$b $(CSED_NATIVE_SO=$R/ab/${v}_C.so py 100 python bench.py --global-batch $b --steps 3000 --warmup 300 --no-epoch $AB_ARGS 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> $O/${T}_ab.log || return 1
  done; done; done
}

task_abtile() {  # same-box A/B of ab/A_C.so vs ab/B_C.so on the large-batch step (B = 1024 / 8192 fp16)
  cd $R && rm -f $O/${T}_abtile.log && \
  for i in $(seq ${N_AB:-3}); do for v in A B; do
    echo "$v B=1024 $(CSED_NATIVE_SO=$R/ab/${v}_C.so py 100 python bench.py --global-batch 1024 --dtype fp16 --steps 400 --warmup 40 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> $O/${T}_abtile.log || return 1
    echo "$v B=8192 $(CSED_NATIVE_SO=$R/ab/${v}_C.so py 100 python bench.py --global-batch 8192 --dtype fp16 --steps 60 --warmup 6 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> $O/${T}_abtile.log || return 1
  done; done
}

task_abcfg() {  # same-box A/B of ab/A_C.so vs ab/B_C.so over AB_CFGS (';'-separated bench argument sets)
  cd $R && rm -f $O/${T}_abcfg.log && \
  IFS=';' read -ra CFGS <<< "${AB_CFGS:---global-batch 64 --steps 3000 --warmup 300;--global-batch 8 --loopback-world 8 --steps 3000 --warmup 300;--global-batch 1024 --dtype fp16 --steps 400 --warmup 40;--global-batch 8192 --dtype fp16 --steps 60 --warmup 6}" && \
  for i in $(seq ${N_AB:-3}); do for c in "${CFGS[@]}"; do for v in A B; do
    echo "$v [$c] $(CSED_NATIVE_SO=$R/ab/${v}_C.so py 100 python bench.py $c --no-epoch --no-fp32-record 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> $O/${T}_abcfg.log || return 1
  done; done; done
}

task_pmctile() {
  pmc3 ${T}_pmc1024 1024 100
}

task_abenv() {
  cd $R && rm -f $O/${T}_abenv.log && \
  for i in $(seq ${N_AB:-3}); do for v in A B; do
    if [ $v = A ]; then E="$ENV_A"; else E="$ENV_B"; fi
    echo "$v $(env $E timeout -k 10 100 python bench.py ${BENCH_ARGS:---steps 3000 --warmup 300 --no-epoch} $AB_ARGS 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> $O/${T}_abenv.log || return 1
  done; done
}

task_splitk() {
  cd /tmp && export TMPDIR=/tmp && \
  for i in 1 2; do for v in A B; do
    CSED_NATIVE_SO=$R/ab/${v}_C.so py 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_splitk_${v}$i -o run -- python3 $R/bench.py --global-batch 8192 --dtype fp16 --steps 60 --warmup 6 --no-epoch --no-fp32-record > $O/${T}_splitk_${v}$i.log 2>&1 || return 1
  done; done && \
  cd $R && py 400 python -u tools/loopback_soak.py --rounds 20 > $O/${T}_soak.log 2>&1
}

task_ipcmem() {
  cd $R && CSED_IPC_MEM=finegrained py 300 python -u -m pytest tests/test_exchange_loopback_gpu.py tests/test_comm_gpu.py -v --timeout 200 --timeout-method thread > $O/${T}_tests_fine.log 2>&1 && \
  py 200 python -u tools/exchange_trace.py --batch 8 32 --worlds 1 2 8 > $O/${T}_trace_uncached.log 2>&1 && \
  CSED_IPC_MEM=finegrained py 200 python -u tools/exchange_trace.py --batch 8 32 --worlds 1 2 8 > $O/${T}_trace_fine.log 2>&1
}

task_epoch0() {
  cd $R && py 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_e0_driver.json 2>$O/${T}_e0_driver.err && \
  py 200 python bench.py --gpus 1 --steps 20 --warmup 5 --epoch0-stamps > $O/${T}_e0_stamps.json 2>$O/${T}_e0_stamps.err && \
  py 200 python bench.py --gpus 1 --steps 20 --warmup 5 --dtype fp32 --epoch0-stamps > $O/${T}_e0_fp32.json 2>$O/${T}_e0_fp32.err && \
  CSED_PRELOAD=1 py 200 python bench.py --gpus 1 --steps 20 --warmup 5 --epoch0-stamps > $O/${T}_e0_preload.json 2>$O/${T}_e0_preload.err && \
  py 120 python tools/firstlaunch_probe.py > $O/${T}_e0_probe.json 2>$O/${T}_e0_probe.err && \
  py 120 python tools/firstlaunch_probe.py --preload > $O/${T}_e0_probe_pre.json 2>$O/${T}_e0_probe_pre.err && \
  py 200 python bench.py --gpus 1 --steps 20 --warmup 5 --epoch0-stamps > $O/${T}_e0_stamps2.json 2>$O/${T}_e0_stamps2.err
}

task_bringtrace() {  # HIP-API + kernel + copy trace of the bench's bring-up (tools/bringup_trace.py)
  cd /tmp && export TMPDIR=/tmp && \
  py 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/${T}_bt -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-fp32-record --no-epoch > $O/${T}_bt.log 2>&1 && \
  cd $R && python3 tools/bringup_trace.py $O/${T}_bt --min-ms 0.3 > $O/${T}_bt_summary.txt 2>&1
}

task_graphab() {  # native HipGraph vs torch.cuda.CUDAGraph step graphs, alternating (driver command + long window;
                 # GRAPH_AB: native nativeflags nativeupload torch)
  cd $R && rm -f $O/${T}_graphab.log && \
  for i in 1 2 3; do for v in ${GRAPH_AB:-native torch}; do
    case $v in native) E=CSED_NATIVE_GRAPH=1;; nativeflags) E="CSED_NATIVE_GRAPH=1 CSED_GRAPH_FLAGS=1";; nativeupload) E="CSED_NATIVE_GRAPH=1 CSED_GRAPH_UPLOAD=1";;
      stream) E=CSED_BENCH_STREAM=1;; nativestream) E="CSED_NATIVE_GRAPH=1 CSED_BENCH_STREAM=1";; *) E=CSED_NATIVE_GRAPH=0;; esac
    echo "$v driver $(env $E timeout -k 10 100 python bench.py --gpus 1 --steps 20 --warmup 5 --no-fp32-record 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["time_elapsed_s"], d["epoch_s"])')" >> $O/${T}_graphab.log || return 1
    echo "$v long $(env $E timeout -k 10 100 python bench.py --steps 3000 --warmup 300 --no-epoch --no-fp32-record 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])')" >> $O/${T}_graphab.log || return 1
  done; done
}

task_diag() {  # the data-parallel diagnostics: rejected-exchange benches, dpcheck rehearsal (2 gloo ranks)
  cd $R && py 600 python -u -m pytest tests/test_fault_injection_gpu.py tests/test_multigpu_gpu.py -v --timeout 300 --timeout-method thread > $O/${T}_diag_tests.log 2>&1 && \
  py 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29531 -m csed_514_project_distributed_training_using_pytorch_amd.parallel.dpcheck --backend gloo --steps 8 > $O/${T}_dpcheck2.log 2>&1
}

task_conv4096() {  # the per-op conv kernels at large batch: fusion tests, B = 4096 step times, phase-split trace
  cd $R && py 600 python -u -m pytest tests/test_modular_fusion_gpu.py tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread > $O/${T}_convtests.log 2>&1 && \
  py 300 python -u tools/ddp_overlap.py --batch 4096 --steps 50 --graph graph > $O/${T}_mod4096.log 2>&1 && \
  CSED_UNPOOL_MIN_BATCH=1000000 py 300 python -u tools/ddp_overlap.py --batch 4096 --steps 50 --graph graph > $O/${T}_mod4096_fusedpool.log 2>&1 && \
  py 300 python -u tools/conv_stamps.py --batch 4096 > $O/${T}_convstamps4096.log 2>&1 && \
  cd /tmp && py 300 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_modkt4096 -o run -- python3 $R/tools/ddp_overlap.py --trace --batch 4096 --mode nocomm --bucket-mb 25 --graph graph > $O/${T}_modkt4096.log 2>&1 && \
  cd $R && python3 tools/ddp_overlap.py --phases $(ls $O/${T}_modkt4096/*kernel_trace.csv $O/${T}_modkt4096/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/${T}_modkt4096_phases.json 2>&1
}

task_modsteps() {  # the modular step at B = 64 and 4096: per-op launch times and graph step times
  cd $R && py 200 python -u tools/op_probe.py --batch 64 > $O/${T}_op64.log 2>&1 && \
  py 300 python -u tools/op_probe.py --batch 4096 --reps 20 > $O/${T}_op4096.log 2>&1 && \
  py 300 python -u tools/ddp_overlap.py --batch 64 --graph graph > $O/${T}_mod64.log 2>&1 && \
  py 300 python -u tools/ddp_overlap.py --batch 4096 --graph graph --only single:25 --loader > $O/${T}_mod4096_loader.log 2>&1 && \
  py 300 python -u tools/ddp_overlap.py --batch 64 --graph graph --only single:25 --loader > $O/${T}_mod64_loader.log 2>&1
}

task_wgradab() {  # same-build A/B of the weight-gradient staging depth (CSED_WGRAD_PF=1 vs the built depth)
  cd $R && rm -f $O/${T}_wgradab.log && \
  for i in $(seq ${N_AB:-3}); do for v in 1 2; do
    echo "PF=$v" >> $O/${T}_wgradab.log && \
    CSED_WGRAD_PF=$v py 300 python -u tools/op_probe.py --batch 4096 --reps 20 2>/dev/null | grep -E "conv[12] bwd" >> $O/${T}_wgradab.log && \
    CSED_WGRAD_PF=$v py 300 python -u tools/ddp_overlap.py --batch 4096 --graph graph --only single:25 2>/dev/null | tail -2 >> $O/${T}_wgradab.log || return 1
  done; done
}

task_quick() {  # the test files this round's changes touch
  cd $R && py 600 python -u -m pytest tests/test_modular_fusion_gpu.py tests/test_modular_graph_gpu.py tests/test_fused_gpu.py tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread > $O/${T}_quick.log 2>&1
}

for task in ${TASKS//,/ }; do
  echo "[gpu.sh] $task $(date +%T)"
  task_$task || { echo "[gpu.sh] $task failed rc=$?"; exit 1; }
done
echo "[gpu.sh] done"
