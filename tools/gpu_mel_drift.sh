# Log-mel drift under a concurrent encoder: default library, then the variant with
# packed FP32 in mel.o only.  usage: gpu_mel_drift.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-meld}; mkdir -p $O
timeout -k 10 200 python -u tools/mel_drift_probe.py none encode layer > $O/mel_default.txt 2>&1
OSW_LIB=$PWD/open-speech_amd/lib/libosw_hip_pk_mel.so timeout -k 10 200 python -u tools/mel_drift_probe.py none encode layer > $O/mel_pk.txt 2>&1
