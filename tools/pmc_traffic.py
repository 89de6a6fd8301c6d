"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <workload> [out.json]

Reads each pass's *counter_collection.csv, groups dispatches by the category
bench.py's live timer reports (sd_prof names), and stores per category the
mean HBM bytes per launch = 2 x FETCH_SIZE (gfx950 tallies a 128-B streaming
read request as 64 B, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KiB
units as rocprofv3 reports them.  bench.py copies [workload][kernel] into
roofline.traffic.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

# sd_prof category -> HIP kernel symbols dispatched under it.
CATEGORIES = {
    # rowprog.hip programs are separate instantiations: <TT, PROBE, PROG> (PROG: bit 0 pre-GEMM, bits 1-2 FFNs)
    "rowprog_out": r"rowprog_kernel<1, 0, 1>",
    "rowprog_ffn": r"rowprog_kernel<1, 0, 2>",
    "rowprog_pw2_ffn": r"rowprog_kernel<1, 0, [35]>",
    "mha_block": r"mha_block_kernel",
    "fcm_stem": r"fcm_conv3x3_band_kernel<2, 2, true",
    "gemm_ring": r"gemm_ring_kernel",
    "gemm_stream": r"gemm_stream_kernel",
    "gemm_areg": r"gemm_areg_kernel",
    "gemm_dma": r"gemm_dma_kernel",
    "gemm_bf16_reg": r"gemm_bf16_kernel",
    "fcm_conv3x3_band": r"fcm_conv3x3_kernel|fcm_conv3x3_band_kernel<(4, 1|2, 2|10, 2), false|fcm_conv3x3_ring_kernel",
    "attention_bf16": r"attn_\w*kernel|attention\w*kernel",
    "lstm_recurrence": r"lstm_(?!handoff|granule)\w*kernel",   # not the hand-off floor probes
    "dwconv": r"glu_dwconv_kernel|dwconv_pk_kernel|dwconv_pp_kernel",
    "groupnorm_silu": r"groupnorm\w*kernel",
    "cam_context": r"cam_context\w*kernel",
    "cam_dense": r"cam_dense_kernel",
    "fbank_kaldi": r"fbank\w*kernel",
}


def _base(name):
    """Kernel symbol without its argument list."""
    return name.replace("(anonymous namespace)", "").split("(")[0]


def _read(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(lambda: [0.0, 0])   # kernel name -> [sum, dispatches]
    csv.field_size_limit(1 << 30)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                p = per[row["Kernel_Name"]]
                p[0] += float(row["Counter_Value"])
                p[1] += 1
    return per


def main():
    fetch_dir, write_dir, workload = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    fetch, write = _read(fetch_dir, "FETCH_SIZE"), _read(write_dir, "WRITE_SIZE")
    res, detail = {}, {}
    for cat, pat in CATEGORIES.items():
        rx = re.compile(pat)
        fk = [k for k in fetch if rx.search(_base(k))]
        wk = [k for k in write if rx.search(_base(k))]
        n = sum(fetch[k][1] for k in fk)
        if not n:
            continue
        f_kib = sum(fetch[k][0] for k in fk)
        w_kib = sum(write[k][0] for k in wk)
        nw = sum(write[k][1] for k in wk)
        bytes_per_launch = (2 * f_kib / n + (w_kib / nw if nw else 0.0)) * 1024
        res[cat] = round(bytes_per_launch)
        detail[cat] = dict(launches=n, fetch_size_kib_per_launch=f_kib / n,
                           write_size_kib_per_launch=w_kib / nw if nw else None,
                           hbm_bytes_per_launch=bytes_per_launch, kernels=sorted({_base(k) for k in fk}))
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[workload] = res
    data.setdefault("_detail", {})[workload] = detail
    with open(out, "w") as f:
        json.dump(data, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
