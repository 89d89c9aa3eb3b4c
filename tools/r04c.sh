set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 120 ./tools/probe/chain_write_probe 3600 > gpurun_out/r04c/chain_write_probe.txt 2>&1
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg2 --reps 6 --steps 300 --variants '[{}, {"overlap_min_bytes": 0}]' > gpurun_out/r04c/ab_cfg2.json 2> gpurun_out/r04c/ab_cfg2.log
