# round 6: the patch embedding as one whole-batch launch on stream 0 before the fork
# (NQK_EMBED_WHOLE=1) against the two half-batch launches on two streams, interleaved, ViT-Base and ViT-Ti
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --no-secondary --steps 30 --warmup 3"
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r6l_main_$r.json 2>gpurun_out/r6l_main_$r.err || exit 4
  NQK_EMBED_WHOLE=1 timeout -k 10 200 python -u bench.py $A > gpurun_out/r6l_whole_$r.json 2>gpurun_out/r6l_whole_$r.err || exit 5
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py $A --config vit_tiny > gpurun_out/r6l_tiny_main_$r.json 2>gpurun_out/r6l_tiny_main_$r.err || exit 6
  NQK_EMBED_WHOLE=1 timeout -k 10 200 python -u bench.py $A --config vit_tiny > gpurun_out/r6l_tiny_whole_$r.json 2>gpurun_out/r6l_tiny_whole_$r.err || exit 7
done
rm -rf gpurun_out/r6l_prof
NQK_EMBED_WHOLE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6l_prof -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/r6l_prof.json 2>gpurun_out/r6l_prof.err || exit 8
echo done > gpurun_out/r6l_status.txt
