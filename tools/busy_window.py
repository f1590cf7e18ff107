import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),r["Kernel_Name"]) for r in csv.DictReader(open(f)))
# last 40% of the run
n=len(rows); R=rows[int(n*0.6):]
t0=R[0][0]; t1=max(e for _,e,_ in R)
busy=0; cur_s=None; cur_e=None
for s,e,_ in R:
    if cur_e is None or s>cur_e:
        if cur_e is not None: busy+=cur_e-cur_s
        cur_s,cur_e=s,e
    else: cur_e=max(cur_e,e)
busy+=cur_e-cur_s
print(f"window {(t1-t0)/1e3:.0f} us, busy {busy/1e3:.0f} us ({100*busy/(t1-t0):.1f}%), kernels {len(R)}")
