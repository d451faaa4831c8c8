# summarise tools/pipe_ab.sh output: replay / total per pipeline and library
for tag in $TAGS; do for p in $PIPES; do python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/pipe_${tag}_$p/run_kernel_stats.csv')))
tot=sum(float(x['TotalDurationNs']) for x in rows if x['Name'].startswith(('bq','void bq')))/3/1e6
top=sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:3]
print('%-18s %-14s bq total/iter %.3f ms |' % ('$tag', '$p', tot), ' '.join('%s=%.0f' % (r['Name'].split('(')[0].replace('void bq::','')[:26], float(r['TotalDurationNs'])/3000) for r in top))
"; done; done
