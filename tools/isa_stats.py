"""Static instruction mix of a kernel per s_barrier-delimited region (VALU, lane
read/writes (SGPR spills), transcendentals, LDS, MFMA, SALU, VMEM), from hipcc
--save-temps assembly.  Usage: python tools/isa_stats.py <file.s> <mangled kernel name>"""
import re,sys
S=open(sys.argv[1]).read().split("\n")
name=sys.argv[2]
start=[i for i,l in enumerate(S) if l.startswith(name+":")][0]
regions=[[]]
for l in S[start+1:]:
    if l.startswith("\ts_endpgm"): break
    t=l.strip()
    if not t or t.startswith(";") or t.startswith("."): continue
    regions[-1].append(t)
    if t.startswith("s_barrier"): regions.append([])
for i,r in enumerate(regions):
    ops=[x.split()[0] for x in r]
    valu=sum(1 for o in ops if o.startswith("v_") and not o.startswith("v_mfma") and not o.startswith("v_readlane") and not o.startswith("v_writelane"))
    rl=sum(1 for o in ops if o.startswith("v_readlane") or o.startswith("v_writelane") or o.startswith("v_readfirstlane"))
    trans=sum(1 for o in ops if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_",o))
    ds=sum(1 for o in ops if o.startswith("ds_"))
    mf=sum(1 for o in ops if o.startswith("v_mfma"))
    sa=sum(1 for o in ops if o.startswith("s_"))
    vm=sum(1 for o in ops if o.startswith("global_") or o.startswith("buffer_"))
    print(f"region {i:2d}: total {len(ops):5d} valu {valu:4d} lane-rw {rl:3d} trans {trans:3d} ds {ds:4d} mfma {mf:3d} salu {sa:4d} vmem {vm:3d}")
