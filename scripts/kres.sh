#!/bin/bash
# Register / scratch usage of the query kernels in a built object: kres.sh build/obj/kernels_tu2.o [name filter]
set -e
o=$1; f=${2:-.}
t=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$t/fb $o
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$t/fb --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $t/co | python3 -c "
import sys,re
cur={}
out=[]
for line in sys.stdin:
    m=re.match(r'\s+\.(name|vgpr_count|sgpr_count|private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count|agpr_count|group_segment_fixed_size):\s+(\S+)',line)
    if m:
        k,v=m.groups()
        if k=='name' and not v.endswith('.kd'):
            cur={'name':v}; out.append(cur)
        elif k!='name' and out: out[-1][k]=v
for d in out:
    if re.search('$f', d.get('name','')):
        print(d.get('name')[:90], 'vgpr',d.get('vgpr_count'),'agpr',d.get('agpr_count'),'sgpr',d.get('sgpr_count'),'scratch',d.get('private_segment_fixed_size'),'vspill',d.get('vgpr_spill_count'),'sspill',d.get('sgpr_spill_count'))
"
rm -rf $t
