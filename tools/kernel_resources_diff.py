#!/usr/bin/env python3
"""Per-kernel VGPR / spill / occupancy of a HIP source against another version of it
(hipcc -Rpass-analysis=kernel-resource-usage); prints only the kernels that differ.
usage: kernel_resources_diff.py OLD.hip NEW.hip  (paths relative to open-speech_amd/csrc)"""
import re,sys,subprocess
def res(src):
    out=subprocess.run(["/opt/rocm/bin/hipcc","--offload-arch=gfx950","-O3","-std=c++17","-fPIC","-munsafe-fp-atomics","-Xclang","-target-feature","-Xclang","-packed-fp32-ops","--offload-device-only","-c",src,"-o","/tmp/x.o","-Rpass-analysis=kernel-resource-usage"],capture_output=True,text=True,cwd="/root/repo/open-speech_amd/csrc").stderr
    d={};cur=None
    for l in out.splitlines():
        m=re.search(r"Function Name: (\S+)",l)
        if m: cur=m.group(1); d[cur]={}; continue
        m=re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)",l)
        if m and cur: d[cur][m.group(1)]=int(m.group(2))
    return d
a=res(sys.argv[1]); b=res(sys.argv[2])
for k in sorted(set(a)|set(b)):
    if a.get(k)!=b.get(k): print(k[:90], a.get(k), '->', b.get(k))
