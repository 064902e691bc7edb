"""Register / spill summary of the render kernel instances in a hipcc -S listing (amdhsa metadata):
   python tools/regs.py file.s  -> one line per render_kernel instance"""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r"\.name:\s+(_ZN3crt3dev1[0-9](?:render|hits)\w+)\n(.*?)(?=\n  - |\n\.end_amdgpu_metadata)", s, re.S):
    name, body = m.group(1), m.group(2)
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", body))
    short = re.sub(r"_ZN3crt3dev13render_kernelI(\w)Lb(\d)ELb(\d)ELb(\d)ELi(\d)ELb(\d)E.*", r"SE=\1 GSTACK=\2 LSCENE=\3 COUNT=\4 PM=\5 W5=\6", name)
    print(f"{short:48s} vgpr {f.get('vgpr_count'):>4} spill {f.get('vgpr_spill_count'):>3} sgpr_spill {f.get('sgpr_spill_count'):>3} scratch {f.get('private_segment_fixed_size'):>4}")
