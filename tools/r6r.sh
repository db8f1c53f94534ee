# round 6: is k_pg's time linear in its tiles, or does the partial last pass of the persistent grid cost?
# FFN-down / FFN-up / out-proj at M giving 2.0, 2.31 (ViT-Base B = 256) and 3.0 tiles per workgroup slot
set -u
mkdir -p gpurun_out
for m in 43690 50432 65536; do
  GM_M=$m PGM_SHAPES=out,up,down PGM_ROUNDS=3 timeout -k 10 300 python -u tools/pg_micro.py > gpurun_out/r6r_m$m.txt 2>&1 || exit 3
done
echo done > gpurun_out/r6r_status.txt
