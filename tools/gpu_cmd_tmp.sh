set -o pipefail
for w in 512 256 384 768 1024 512; do GNNEA_X3TA_WGS=$w timeout -k 10 100 python tools/dbg/x3ta.py 2>&1 | grep -v amdgpu.ids || exit 1; done
