#!/bin/bash
# Copy a tools/gpu_r04_final.sh run's results from gpurun_out/ into profiles/ under round tag $1
# (e.g. r04): bench lines, kernel stats, PMC summaries, GPU test tail, rehearsal, configs, syn A/B.
set -e
T=${1:?round tag}; O=gpurun_out; P=profiles
tail -1 $O/bench.log > $P/${T}_bench.json
tail -1 $O/bench_c4.log > $P/${T}_bench_c4_n1.json
tail -1 $O/bench_c5.log > $P/${T}_bench_c5_n1.json
cp $O/prof/run_kernel_stats.csv $P/${T}_kernel_stats.csv
cp $O/prof_c4/run_kernel_stats.csv $P/${T}_kernel_stats_c4.csv
cp $O/prof_c5/run_kernel_stats.csv $P/${T}_kernel_stats_c5.csv
for W in c2 c4 c5; do cp $O/pmc_$W.json $P/pmc_$W.json; done
tail -5 $O/pytest_gpu.log > $P/${T}_pytest_gpu_tail.log
tail -1 $O/smoke.log >> $P/${T}_pytest_gpu_tail.log
grep '^{' $O/rehearse.log > $P/${T}_rehearse_gpus2_one_gpu_gloo.jsonl
cp $O/configs.json $P/${T}_configs.json
cp $O/syn_ab_final.jsonl $P/${T}_syn_ab_final.jsonl
