"""Summarise tools/pmc_sq.sh output: per kernel, counter sums per dispatch."""
import csv, glob, sys
from collections import defaultdict

def load(d):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for row in csv.DictReader(open(f)):
            k = row['Kernel_Name'].split('(')[0]
            acc[k][row['Counter_Name']] += float(row['Counter_Value'])
            disp[k].add((f, row['Dispatch_Id']))
    return acc, disp

acc, disp = load(sys.argv[1])
for k, c in acc.items():
    n = max(1, len({d for d in disp[k]}) // 3)
    print(k, 'dispatches/pass', n)
    for name in sorted(c):
        print('   %-26s %16.0f' % (name, c[name] / n))
