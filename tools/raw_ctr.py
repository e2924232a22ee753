import csv, collections, glob, sys
d=sys.argv[1]
tot=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.defaultdict(set)
for f in glob.glob(d+'/*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        k=r['Kernel_Name']
        if 'classattn' not in k: continue
        tot[(k[:60],f.split('/')[-2])][r['Counter_Name']]+=float(r['Counter_Value']); n[(k[:60],f.split('/')[-2])].add(r['Dispatch_Id'])
for (k,f),c in sorted(tot.items()):
    nd=len(n[(k,f)])
    print(k, f, {a: '%.3g'%(v/nd) for a,v in c.items()})
