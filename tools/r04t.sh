set -o pipefail
mkdir -p gpurun_out/r04t
timeout -k 10 600 python -u tools/ab_opts.py --workload cfg3 --reps 3 --steps 200 --variants '[{}, {"chain_words": 6144}, {"chain_words": 12288}, {"chain_max": 5}, {"chain_max": 3}, {"launch_bytes": 8000000}, {"launch_bytes": 32000000}, {"pad_words": 8}]' > gpurun_out/r04t/ab_cfg3.json 2> gpurun_out/r04t/ab_cfg3.log
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg4 --reps 3 --steps 100 --variants '[{}, {"chain_words": 12288}, {"chain_max": 5}, {"chain_waves": 16}]' > gpurun_out/r04t/ab_cfg4.json 2> gpurun_out/r04t/ab_cfg4.log
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg2 --reps 3 --steps 2000 --variants '[{}, {"chain_words": 12288}, {"chain_waves": 16}, {"chain_waves": 8}]' > gpurun_out/r04t/ab_cfg2.json 2> gpurun_out/r04t/ab_cfg2.log
