#!/bin/bash
# resource usage of the search kernels (device-only compile): SGPR/VGPR counts and
# spills per instantiation.  usage: tools/kres.sh [source.hip] [regex]
SRC=${1:-hsa_amd/csrc/hsa_search.hip}; X=${KRES_FLAGS:-}   # KRES_FLAGS: extra -D flags
RE=${2:-k_search|k_widths}
cd "$(dirname "$0")/.." || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only $X -S "$SRC" -o /tmp/kres.s 2>/dev/null || exit 1
python3 - "$RE" <<'PY'
import re, sys
s = open('/tmp/kres.s').read()
for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)\.wavefront_size', s, re.S):
    name, body = m.group(1), m.group(2)
    if not re.search(sys.argv[1], name):
        continue
    g = lambda k: re.search(k + r':\s+(\d+)', body).group(1)
    fn = re.search(r'\n' + re.escape(name) + r':(.*?)s_endpgm', s, re.S)
    n = sum(1 for l in fn.group(1).split('\n') if l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;')) if fn else -1
    print(f"{name[:60]:60s} sgpr {g('sgpr_count'):>3} spill {g('sgpr_spill_count'):>3}  vgpr {g('vgpr_count'):>3} spill {g('vgpr_spill_count'):>3}  insts {n}")
PY
