set -o pipefail
mkdir -p gpurun_out/r04q
timeout -k 10 400 python -u tools/ab_opts.py --workload cfg2 --reps 3 --steps 2000 --variants '[{"flood": 0}, {"flood": 0, "chain_max": 6}, {"flood": 0, "chain_max": 3}, {"flood_top_bytes": 200000}, {"flood": 0, "launch_bytes": 4000000}, {"flood": 0, "launch_bytes": 64000000}]' > gpurun_out/r04q/ab_cfg2b.json 2> gpurun_out/r04q/ab_cfg2b.log
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg3 --reps 3 --steps 200 --variants '[{}, {"flood": 0}]' > gpurun_out/r04q/ab_cfg3.json 2> gpurun_out/r04q/ab_cfg3.log
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg4 --reps 3 --steps 100 --variants '[{}, {"flood": 0}]' > gpurun_out/r04q/ab_cfg4.json 2> gpurun_out/r04q/ab_cfg4.log
