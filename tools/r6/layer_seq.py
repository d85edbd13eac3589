import csv, sys, collections
# per-dispatch sequence of conv kernels in one steady step: (order index, short name, grid, us)
def load(f, steps=5):
    rows=[r for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r:int(r['Start_Timestamp']))
    # group into steps by a marker kernel: adam_kernel occurrences (2 per step)
    idx=[i for i,r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
    # last full step: between adam #-4 and #-2 (2 adam per step)
    a,b=idx[-5],idx[-1]
    out=[]
    for r in rows[a+1:b+1]:
        n=r['Kernel_Name']
        if 'conv' in n and ('fwd' in n or 's2t' in n or 'halo' in n):
            out.append((n.split('(')[0].replace('void p2p::','')[:60], r['Grid_Size_X'], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000))
    return out
A=load(sys.argv[1]); B=load(sys.argv[2])
print(len(A),len(B))
for x,y in zip(A,B):
    print(f"{x[0]:60s} {x[1]:>8s} {x[2]:8.1f} | {y[0]:60s} {y[1]:>8s} {y[2]:8.1f}")
