"""HBM bytes per k_env_step launch from the FETCH_SIZE / WRITE_SIZE passes of run_profile.sh.

Usage: python profiles/traffic_from_pmc.py <fetch counter csv> <write counter csv> <alg bytes> <out.json> [variant]
       [kernel] [rounds per launch]
kernel: k_env_step (default) or k_env_rollout_act_free, whose one launch runs [rounds per launch] rounds: its
bytes are then reported per round (alg bytes: per round), the unit of the bench's roofline for it.

Both counters are in KiB per dispatch. Per MI355X_MICROARCH.md § HBM: FETCH_SIZE reports half
the bytes of a wide coalesced read on gfx950 (doubled here); WRITE_SIZE is exact for 16-byte
streaming stores (the observation / record / reward stores of the kernel). The result is the
average over the profiled launches; bench.py reads it as roofline.traffic.
"""
import csv
import datetime
import json
import sys


def per_launch(path, counter, kernel="k_env_step"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    assert vals, "no %s %s rows in %s" % (kernel, counter, path)
    return sum(vals) / len(vals) * 1024.0, len(vals)


def main():
    fetch_csv, write_csv, alg, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    variant = sys.argv[5] if len(sys.argv) > 5 else ""
    kernel = sys.argv[6] if len(sys.argv) > 6 else "k_env_step"
    rounds = int(sys.argv[7]) if len(sys.argv) > 7 else 1
    fetch, nf = per_launch(fetch_csv, "FETCH_SIZE", kernel)
    write, nw = per_launch(write_csv, "WRITE_SIZE", kernel)
    fetch, write = fetch / rounds, write / rounds
    total = 2.0 * fetch + write
    d = {"kernel": kernel, "rounds_per_launch": rounds, "bytes": total, "fetch_bytes_raw": fetch,
         "fetch_bytes_corrected": 2.0 * fetch,
         "write_bytes": write, "launches": [nf, nw], "algorithmic_bytes": alg, "vs_algorithmic": total / alg,
         "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE as reported; KiB -> bytes",
         "variant": variant,
         # bench.py's committed_traffic picks the newest measurement of a workload by this stamp
         "measured_at": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds")}
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
