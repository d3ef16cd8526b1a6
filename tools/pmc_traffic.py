"""HBM traffic per inflate-pipeline launch from rocprofv3 PMC passes.

Reads the FETCH_SIZE and WRITE_SIZE counter_collection.csv files written by
tools/pmc_traffic.sh (one counter per pass: they do not fit one TCC pass on
gfx950) and applies the gfx950 corrections of MI355X_MICROARCH.md "HBM":
FETCH_SIZE/WRITE_SIZE are in KiB; FETCH_SIZE reports half the bytes of wide
streaming reads, so it is doubled.  Our kernels also issue narrower accesses
(4-byte input words, 2-byte table entries) whose tally is uncalibrated: the
figure is an estimate of bytes crossing the L2's memory side (Infinity Cache
hits included), per launch of each pipeline kernel, averaged over dispatches.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [CHECKPOINT_TAG]
The output records the sha256 of the library the passes ran and the source
hash it was built from (zs_source_hash), so bench.py can say whether the
traffic figure belongs to the sources of the build it is timing.
"""
import csv, ctypes, hashlib, json, os, sys
from collections import defaultdict

PIPELINE = ("zs_header_kernel", "zs_find_kernel", "zs_find_fixed_kernel", "zs_plan_kernel", "zs_unit_header_kernel",
            "zs_unit_keys_kernel", "zs_lane_kernel", "zs_unitw_kernel", "zs_walk_kernel", "zs_split_kernel",
            "zs_unitw_list_kernel", "zs_chain_kernel", "zs_expand_kernel", "zs_expand2_kernel",
            "zs_link_kernel", "zs_linkseg_kernel", "zs_linkseg_join_kernel", "zs_link64_kernel", "zs_plink_init_kernel", "zs_plink_step_kernel", "zs_plink_out_kernel",
            "zs_emit_kernel", "zs_emit64_kernel", "zs_decode_kernel", "zs_check_kernel", "zs_finalize_kernel")


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0.0, set()])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0]
            name = name.replace("void ", "").split("<")[0]
            acc[name][0] += float(row["Counter_Value"])
            acc[name][1].add(row["Dispatch_Id"])
    return {k: (v[0] * 1024.0 / len(v[1]), len(v[1])) for k, v in acc.items()}


def source_hash(so):
    """the source hash the library was built from (zs_source_hash, csrc/srchash.py)"""
    try:
        L = ctypes.CDLL(so)
        L.zs_source_hash.restype = ctypes.c_char_p
        return L.zs_source_hash().decode()
    except (OSError, AttributeError):
        return None


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    kernels = {}
    total = 0.0
    for k in PIPELINE:
        if k not in fetch and k not in write:
            continue
        rd = 2.0 * fetch.get(k, (0.0, 0))[0]
        wr = write.get(k, (0.0, 0))[0]
        kernels[k] = {"read_bytes": round(rd), "write_bytes": round(wr),
                      "dispatches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
        total += rd + wr
    so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zlib-streams_amd", "libzstreams_mi355x.so")
    out = {"hbm_bytes_per_launch": round(total), "kernels": kernels,
           "checkpoint": sys.argv[4] if len(sys.argv) > 4 else None,
           "library_sha256": hashlib.sha256(open(so, "rb").read()).hexdigest(),
           "source_sha256": source_hash(so),
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes); bytes = 2*FETCH_SIZE*1024 "
                     "+ WRITE_SIZE*1024 per dispatch, averaged over dispatches, summed over pipeline kernels"}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
