set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 400 python -u tools/ab_opts.py --workload cfg3 --reps 4 --steps 200 --variants '[{}, {"chain_nt": 0}, {"chain_words": 4096}, {"chain_words": 16384}, {"chain_words": 4096, "chain_nt": 0}, {"chain_max": 5}]' > gpurun_out/r04d/ab_cfg3.json 2> gpurun_out/r04d/ab_cfg3.log
