set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fill
cd /tmp && export TMPDIR=/tmp
export TB_PHASE_MARKS=$R/gpurun_out/fill/marks.json
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pf_fill -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/fill/bench.log 2>&1
LO=$(python3 -c "import json;m=json.load(open('$TB_PHASE_MARKS'));print([t for n,t in m if n.startswith('step')][0])")
HI=$(python3 -c "import json;m=json.load(open('$TB_PHASE_MARKS'));print([t for n,t in m if n=='end'][0])")
python3 $R/tools/gemm_fill.py $R/gpurun_out/pf_fill/run_kernel_trace.csv $LO $HI > $R/gpurun_out/fill/gemm_fill.txt
python3 - <<'PY' > $R/gpurun_out/fill/gemm_shapes.txt
import csv, collections, os
R=os.environ["GRAFT_REPO_ROOT"]
rows=list(csv.DictReader(open(R+"/gpurun_out/pf_fill/run_kernel_trace.csv")))
c=collections.defaultdict(lambda:[0,0.0])
for r in rows:
    n=r["Kernel_Name"]
    if "Cijk" not in n: continue
    wg=int(r["Grid_Size_X"])//max(1,int(r["Workgroup_Size_X"]))
    mt=n.split("_MT")[1].split("_")[0] if "_MT" in n else "?"
    k=(mt,wg)
    c[k][0]+=1; c[k][1]+=(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e6
for k,v in sorted(c.items(), key=lambda kv:-kv[1][1])[:40]:
    print(f"MT{k[0]:12s} wg {k[1]:6d}  n {v[0]:6d}  {v[1]:9.1f} ms  avg {1000*v[1]/v[0]:8.1f} us")
PY
rm -rf $R/gpurun_out/pf_fill
cat $R/gpurun_out/fill/gemm_fill.txt $R/gpurun_out/fill/gemm_shapes.txt
