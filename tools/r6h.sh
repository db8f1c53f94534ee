# round 6: what the residual epilogue's HBM traffic costs the residual GEMMs (diagnostic builds: wrong results)
set -u
mkdir -p gpurun_out
PGM_SHAPES=out,down PGM_LIBS=noresld=tools/diag/libnqk_d4096.so,nostore=tools/diag/libnqk_d1.so,neither=tools/diag/libnqk_d4097.so timeout -k 10 300 python -u tools/pg_micro.py > gpurun_out/r6h_pg_micro.txt 2>&1 || exit 3
