"""Print / save the kernel summary of a rocprofv3 --stats run (sqlite .db output)."""
import glob, sqlite3, sys

def top(d, out=None, n=8):
    db = glob.glob(d + '/**/*.db', recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name,total_calls,total_duration,average,percentage from top_kernels"))
    lines = ["kernel,calls,total_us,avg_us,pct"]
    for r in rows:
        lines.append('"%s",%d,%.1f,%.1f,%.2f' % (r[0], r[1], r[2], r[3], r[4]))  # durations in us
    for r in rows[:n]:
        print('%-44s %4d %9.2f ms %5.1f%%' % (r[0][:44], r[1], r[3] / 1e3, r[4]))
    if out:
        open(out, 'w').write('\n'.join(lines) + '\n')

if __name__ == '__main__':
    top(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
