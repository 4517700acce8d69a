import csv, sys, collections, json
rows = list(csv.DictReader(open(sys.argv[1])))
g = collections.defaultdict(list)
for r in rows:
    if 'rf_nodes_kernel' in r['Kernel_Name']:
        g[int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = [d for v in g.values() for d in v]
print("all", len(tot), round(sum(tot) / len(tot), 2))
for k in sorted(g):
    v = g[k]; print(k, len(v), round(sum(v) / len(v), 2), round(min(v), 2), round(max(v), 2))
