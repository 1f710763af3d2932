# Which object file's packed-FP32 code drifts under a concurrent encoder?  Each library
# variant has v_pk_*_f32 enabled in exactly one object (libosw_hip_pk_<obj>.so).
# usage: gpu_pk_bisect.sh OUT obj...
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pkb}; mkdir -p $O; shift
for v in "$@"; do
  OSW_LIB=$PWD/open-speech_amd/lib/libosw_hip_pk_$v.so timeout -k 10 200 python -u tools/interference_probe.py encode layer > $O/interference_$v.txt 2>&1
done
