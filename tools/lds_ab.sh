set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "lds or short_xcds" > gpurun_out/lds_parity.log 2>&1 || { tail -30 gpurun_out/lds_parity.log; exit 1; }
tail -3 gpurun_out/lds_parity.log
timeout -k 10 200 python -u tools/tune_sweep.py --configs '[{}, {"lds": 1}, {}, {"lds": 1}]' > gpurun_out/lds_h2.jsonl 2>&1
timeout -k 10 200 python -u tools/tune_sweep.py --halo 1 --configs '[{}, {"lds": 1}, {}, {"lds": 1}]' > gpurun_out/lds_h1.jsonl 2>&1
timeout -k 10 200 python -u tools/emu_rank_bench.py 8 > gpurun_out/lds_emu8_base.jsonl 2>&1
GHX_TUNE=lds=1 timeout -k 10 200 python -u tools/emu_rank_bench.py 8 > gpurun_out/lds_emu8_lds.jsonl 2>&1
