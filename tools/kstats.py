import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 23
print(f"total {tot/1e6:.2f} ms over the trace, {tot/1e3/steps:.1f} us/step (steps={steps:g})")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    print(f"{r['Name'][:58]:58s} calls={r['Calls']:>6} avg_us={float(r['AverageNs'])/1e3:8.1f} "
          f"per_step_us={float(r['TotalDurationNs'])/1e3/steps:8.1f} tot%={float(r['TotalDurationNs'])/tot*100:5.1f}")
