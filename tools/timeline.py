"""Print one bench step's kernel timeline from a rocprofv3 kernel_trace.csv (start/end in us
relative to the step's first kernel, queue id, name). usage: timeline.py trace.csv [step]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    step = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    starts = [i for i, r in enumerate(rows) if "keyprep_decode" in r["Kernel_Name"] and not any("keyprep_decode" in q["Kernel_Name"] for q in rows[max(0, i - 1):i])]
    j = starts[step]
    end = starts[step + 1] if step + 1 < len(starts) and step != -1 else len(rows)
    t0 = int(rows[j]["Start_Timestamp"])
    for r in rows[j:end]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} q{r.get('Queue_Id', '?')} {r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main()
