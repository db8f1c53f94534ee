set -x
nproc; grep -m1 'model name' /proc/cpuinfo; free -g | head -2
python -c "import numpy as np; np.show_runtime()" 2>&1 | head -30
rocminfo 2>&1 | grep -E 'Marketing|gfx|Compute Unit|Max Clock' | head -12
hipcc --version | head -2
ls /opt/rocm/lib/librccl* | head
