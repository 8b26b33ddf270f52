set -e
H1='[{"bwd_handout": 1}, {"bwd_handout": 2}]'
F1='[{"fwd_handout": 1}, {"fwd_handout": 2}]'
for k in 8 16 32 64; do
  timeout -k 10 120 python -u tools/bwd_opts.py --k $k --rounds 5 --opts "$H1"
  timeout -k 10 120 python -u tools/fwd_opts_sweep.py --k $k --rounds 5 --opts "$F1"
done
for k in 8 32; do
  timeout -k 10 120 python -u tools/bwd_opts.py --dataset ogbn-proteins --k $k --rounds 3 --opts "$H1"
done
timeout -k 10 120 python -u tools/shard_time.py --worlds 8 --layouts records --opts '{"bwd_handout": 2}'
timeout -k 10 120 python -u tools/shard_time.py --worlds 8 --layouts records --opts '{"bwd_handout": 1}'
timeout -k 10 120 python -u tools/shard_time.py --worlds 8 --layouts records --opts '{"fwd_handout": 2}'
timeout -k 10 120 python -u tools/shard_time.py --worlds 2,4 --layouts records --opts '{"bwd_handout": 2}'
timeout -k 10 120 python -u tools/shard_time.py --worlds 2,4 --layouts records --opts '{"bwd_handout": 1}'
