"""Print one bench step's kernel timeline from a rocprofv3 kernel_trace.csv (start/end in us
relative to the step's first kernel, queue id, name). usage: timeline.py trace.csv [step]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    step = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    # a step starts at its first key decode; the three families' decodes of one step lie within 5 ms
    starts, last = [], None
    for i, r in enumerate(rows):
        if "keyprep_decode" in r["Kernel_Name"]:
            t = int(r["Start_Timestamp"])
            if last is None or t - last > 5_000_000:
                starts.append(i)
            last = t
    j = starts[step]
    end = starts[step + 1] if step + 1 < len(starts) and step != -1 else len(rows)
    t0 = int(rows[j]["Start_Timestamp"])
    for r in rows[j:end]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} q{r.get('Queue_Id', '?')} {r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main()
