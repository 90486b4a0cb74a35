"""Reduce the traffic-calibration probe's rocprofv3 passes (scripts/probes/traffic_calib.hip) to bytes per
counter unit for each access pattern, and apply it to k_step's own FETCH_SIZE / WRITE_SIZE.

usage: traffic_calib.py <probe_dir_fetch> <probe_dir_write> <probe_json_line> [<kstep_traffic_json>]
Writes one JSON object: per pattern the raw FETCH_SIZE / WRITE_SIZE (KB per dispatch, warm dispatches
only: the first of each kernel's back-to-back series is dropped), the known bytes, and the factor
known / raw; then k_step's traffic re-derived with the k_step-pattern factors."""

import csv
import glob
import json
import sys


def per_kernel(d, counter):
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            disp = out.setdefault(k, {})
            disp[int(r["Dispatch_Id"])] = disp.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    res = {}
    for k, disp in out.items():
        ids = sorted(disp)
        warm = [disp[i] for i in ids[1:]] or [disp[i] for i in ids]
        res[k] = sum(warm) / len(warm)
    return res


def main():
    fdir, wdir, probe = sys.argv[1], sys.argv[2], json.loads(sys.argv[3])
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    known_r, known_w = probe["bytes_read"], probe["bytes_written"]
    names = {"k_pattern<1>": "kstep_pattern_xcd_remap", "k_pattern<0>": "kstep_pattern_identity",
             "k_stream": "stream_16B_per_lane", "k_wonly_field<1>": "write_only_kstep_pattern",
             "k_wonly_rows": "write_only_obs_rows"}
    pats = {}
    for k in fetch:
        tag = next((v for s, v in names.items() if s in k), None)
        if tag is None:
            continue
        fr, wr = fetch[k] * 1024.0, write.get(k, float("nan")) * 1024.0
        if tag.startswith("write_only"):
            kw = probe["wonly_field_bytes"] if tag == "write_only_kstep_pattern" else probe["wonly_rows_bytes"]
            pats[tag] = {"fetch_size_bytes_raw": round(fr), "write_size_bytes_raw": round(wr), "known_read_bytes": 0,
                         "known_write_bytes": kw, "fill_bytes_per_written_byte": round(2.0 * fr / kw, 4),
                         "write_factor": round(kw / wr, 4) if wr else None}
            continue
        pats[tag] = {"fetch_size_bytes_raw": round(fr), "write_size_bytes_raw": round(wr),
                     "known_read_bytes": known_r, "known_write_bytes": known_w,
                     "read_factor": round(known_r / fr, 4) if fr else None,
                     "write_factor": round(known_w / wr, 4) if wr else None}
    out = {"probe": probe, "patterns": pats,
           "method": "scripts/probes/traffic_calib.hip: a known byte count moved with k_step's access pattern "
                     "and with 16-B/lane streaming; rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate "
                     "passes; warm dispatches averaged; factor = known bytes / counter bytes"}
    if len(sys.argv) > 4:
        ks = json.load(open(sys.argv[4]))
        p = pats.get("kstep_pattern_xcd_remap", {})
        rf, wf = p.get("read_factor"), p.get("write_factor")
        if rf and wf:
            rd, wrb = ks["fetch_kb"] * 1024.0 * rf, ks["write_kb"] * 1024.0 * wf
            out["k_step"] = {"num_envs": ks["num_envs"], "fetch_kb_raw": ks["fetch_kb"], "write_kb_raw": ks["write_kb"],
                             "read_bytes_calibrated": round(rd), "write_bytes_calibrated": round(wrb),
                             "traffic_bytes_per_launch": round(rd + wrb)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
