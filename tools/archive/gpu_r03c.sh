set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_stream_gpu.py tests/test_piece_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pt_stream.log 2>&1 || { tail -30 $O/pt_stream.log; exit 1; }
tail -1 $O/pt_stream.log
timeout -k 10 300 python3 -u tools/stream_rate.py --mib 1024 --ab > $O/stream_ab2.json 2> $O/stream_ab2.err || { tail -10 $O/stream_ab2.err; exit 1; }
cat $O/stream_ab2.json
timeout -k 10 400 python3 -u tools/syn_ab.py --cases "zfec(64,96)" --variants "direct@SEC_SYN=0,syn@SEC_SYN=1,ring3@SEC_SYN=1/ring3,ring4@SEC_SYN=1/ring4" > $O/syn_ring.jsonl 2> $O/syn_ring.err || { tail -10 $O/syn_ring.err; exit 1; }
cat $O/syn_ring.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_syn -o run -- python3 tools/syn_ab.py --cases "1MiB x1024, 16 lost" --variants "syn@SEC_SYN=1" --rounds 1 > $O/prof_syn.log 2>&1 || { tail -10 $O/prof_syn.log; exit 1; }
cut -d, -f1-5 $O/prof_syn/run_kernel_stats.csv | head -8
