"""Run the bench workload once through the profiling build and print the
in-kernel counters (zs_kprof.h) as per-phase figures.

usage (GPU box): ZS_LIB=$PWD/zlib-streams_amd/libzstreams_mi355x_prof.so \
                 python3 tools/kprof_run.py [--streams 64] [--out FILE.json]
"""
import argparse, json, os, sys, time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

NAMES = {0: "p_waves", 1: "p_cyc_total", 2: "p_cyc_coop", 3: "p_cyc_steps", 4: "p_cyc_flush", 5: "p_groups",
         6: "p_coop_calls", 7: "p_lane_steps", 8: "p_wave_steps", 9: "p_slow_lit", 10: "p_slow_dist",
         11: "p_cyc_max", 12: "p_cyc_init", 13: "p_refills", 14: "p_busy_waves", 15: "p_cyc_busy",
         16: "e_blocks", 17: "e_cyc_total", 18: "e_rounds", 19: "e_jump_iters", 20: "e_cyc_jump", 21: "e_batches",
         22: "e_cyc_max", 23: "e_cyc_init", 24: "e_jump_rounds", 25: "e_cyc_pre",
         44: "w_cyc_total", 45: "w_cyc_max", 46: "w_wave_steps", 47: "w_cyc_exc", 38: "w_cyc_group", 39: "w_exc",
         40: "s_refill1", 41: "s_lit", 42: "s_refill2", 43: "s_dist",  # split parse: units, cycles, wave-steps, group cycles
         26: "d_blocks", 27: "d_cyc_total", 28: "d_cyc_hist", 29: "d_cyc_build", 30: "d_cyc_hdr", 31: "d_cyc_emit",
         32: "d_cyc_out", 33: "d_chunks",

         48: "l_streams", 49: "l_steps", 50: "l_cyc_succ", 51: "l_cyc_walk", 52: "l_cyc_winwrite", 53: "l_cyc_resolve",
         54: "l_cyc_barrier", 55: "l_markers_sample", 56: "l_cyc_total", 57: "l_cyc_max",
         # finder validation (zs_findval_kernel, round 6: a pool of candidates per wave): waves, refill
         # rounds, cycles in symbol steps, wave-steps, lane-steps (lanes with a live candidate), wave cycles
         58: "fv_waves", 59: "fv_rounds", 60: "fv_cyc_steps", 61: "fv_wave_steps", 62: "fv_lane_steps", 63: "fv_cyc_total"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--stream-mib", type=int, default=64)
    ap.add_argument("--out", default=None)
    ap.add_argument("--deflate", action="store_true", help="also run gzip L6 deflate and report the block kernel")
    a = ap.parse_args()
    import numpy as np
    import corpus
    import zstreams
    raws, comps = corpus.batch(0, a.streams, a.stream_mib << 20, 6, -15, 16, True)
    zstreams.kprof_read(reset=True)
    res = zstreams.inflate_batch([bytes(c) for c in comps], -15, [a.stream_mib << 20] * a.streams)
    c = zstreams.kprof_read(reset=True)
    if a.deflate:  # deflate block-kernel counters (gzip level 6 over the raw streams)
        zstreams.deflate_batch([bytes(r) for r in raws], 31, 6)
        cd = zstreams.kprof_read(reset=True)
        c = list(c)
        for i in range(26, 34):
            c[i] = cd[i]
    if not c:
        sys.exit("no counters: ZS_LIB must point at libzstreams_mi355x_prof.so")
    ok = all(r["ret"] == 1 and bytes(o) == bytes(raws[k]) for k, (o, r) in enumerate(res))
    d = {NAMES[i]: v for i, v in enumerate(c) if i in NAMES}
    # expand2 flush counters in lane-parse slots the split parse leaves unused
    d.update({"x_pieces": c[6], "x_pieces_marked": c[7], "x_pieces_marked_tail": c[8], "x_markers": c[12]})
    # unit headers (zs_unit_header_kernel, dynamic first blocks): cycles by phase
    d.update({"uh_units": c[0], "uh_cyc": c[1], "uh_cyc_pro": c[2], "uh_cyc_lens": c[11], "uh_cyc_lit": c[13],
              "uh_cyc_rest": c[14]})
    w = max(d["p_waves"], 1)
    b = max(d["e_blocks"], 1)
    derived = {
        "ok": ok,
        "parse_cycles_per_wave": d["p_cyc_total"] / w, "parse_cycles_max": d["p_cyc_max"],
        "parse_cycles_per_busy_wave": d["p_cyc_busy"] / max(d["p_busy_waves"], 1),
        "parse_tail_ratio_all_waves": d["p_cyc_max"] / max(d["p_cyc_total"] / w, 1),
        "parse_tail_ratio_busy_waves": d["p_cyc_max"] / max(d["p_cyc_busy"] / max(d["p_busy_waves"], 1), 1),
        "parse_frac_coop": d["p_cyc_coop"] / max(d["p_cyc_total"], 1),
        "parse_frac_steps": d["p_cyc_steps"] / max(d["p_cyc_total"], 1),
        "parse_frac_flush": d["p_cyc_flush"] / max(d["p_cyc_total"], 1),
        "parse_cycles_per_wave_step": d["p_cyc_steps"] / max(d["p_wave_steps"], 1),
        "parse_lane_util": d["p_lane_steps"] / max(64 * d["p_wave_steps"], 1),
        "parse_coop_cycles_per_call": d["p_cyc_coop"] / max(d["p_coop_calls"], 1),
        "parse_slow_lit_per_step": d["p_slow_lit"] / max(d["p_lane_steps"], 1),
        "parse_slow_dist_per_step": d["p_slow_dist"] / max(d["p_lane_steps"], 1),
        "parse_refills_per_step": d["p_refills"] / max(d["p_lane_steps"], 1),
        "expand_cycles_per_block": d["e_cyc_total"] / b, "expand_cycles_max": d["e_cyc_max"],
        "expand_cycles_per_round": d["e_cyc_total"] / max(d["e_rounds"], 1),
        "expand_frac_jump": d["e_cyc_jump"] / max(d["e_cyc_total"], 1),
        "expand_jump_rounds_frac": d["e_jump_rounds"] / max(d["e_rounds"], 1),
        "expand_jump_iters_per_jround": d["e_jump_iters"] / max(d["e_jump_rounds"], 1),
        "expand_frac_init": d["e_cyc_init"] / max(d["e_cyc_total"], 1),
        # zs_expand2_kernel (32 KiB windows): counters per wave; init = token batches, pre = B1..B3
        "expand2_frac_batch": d["e_cyc_init"] / max(d["e_cyc_total"], 1),
        "expand2_frac_pre_spin": d["e_cyc_pre"] / max(d["e_cyc_total"], 1),
        "expand2_frac_spin": d["e_cyc_jump"] / max(d["e_cyc_total"], 1),
        "expand2_spin_rounds_frac": d["e_jump_rounds"] / max(d["e_rounds"], 1),
        "expand2_passes_per_round_max_lane": d["e_jump_iters"] / max(d["e_rounds"], 1),
        "link_cycles_per_step": {k: d[k] / max(d["l_steps"], 1) for k in
                                 ("l_cyc_succ", "l_cyc_walk", "l_cyc_winwrite", "l_cyc_resolve", "l_cyc_barrier",
                                  "l_cyc_total")},
        "link_marker_frac_sample": d["l_markers_sample"] / max(d["l_steps"] * 16 * 32, 1),
        "deflate_block_cycles_per_block": {k: d[k] / max(d["d_blocks"], 1) for k in
                                           ("d_cyc_total", "d_cyc_hist", "d_cyc_build", "d_cyc_hdr", "d_cyc_emit",
                                            "d_cyc_out", "d_chunks")},
        "step_phase_cycles_per_wave_step": {k: d[k] / max(d["p_wave_steps"], 1)
                                            for k in ("s_refill1", "s_lit", "s_refill2", "s_dist")},
        # split parse (zs_walk_kernel / zs_split_kernel): cycles per wave-step
        "walk_cycles_per_step": d.get("w_cyc_total", 0) / max(d.get("w_wave_steps", 0), 1),
        "walk_max_wave_ms_at_2p4ghz": d.get("w_cyc_max", 0) / 2.4e6,
        "walk_exc_cycles_per_step": d.get("w_cyc_exc", 0) / max(d.get("w_wave_steps", 0), 1),
        "walk_group_cycles_per_step": d.get("w_cyc_group", 0) / max(d.get("w_wave_steps", 0), 1),
        "walk_steps_cycles_per_step": d.get("p_cyc_steps", 0) / max(d.get("w_wave_steps", 0), 1),
        "walk_refill_cycles_per_step": d.get("p_cyc_busy", 0) / max(d.get("w_wave_steps", 0), 1),
        "walk_exc_per_step": d.get("w_exc", 0) / max(d.get("w_wave_steps", 0), 1),
        "split_cycles_per_wave_step": d.get("s_lit", 0) / max(d.get("s_refill2", 0), 1),
        # split kernel phases (shares of its wave cycles): unit prologue, sub-unit decode (of which group
        # refill + token stores), the rest (epilogue, unit claims)
        "split_frac_prologue": d.get("p_cyc_flush", 0) / max(d.get("s_lit", 0), 1),
        "split_frac_decode": d.get("p_groups", 0) / max(d.get("s_lit", 0), 1),
        "split_frac_group": d.get("s_dist", 0) / max(d.get("s_lit", 0), 1),
        "split_units": d.get("s_refill1", 0),
        # finder validation pool: lane utilisation, cycles per wave-step, share of the wave's time in steps
        "fv_lane_util": d.get("fv_lane_steps", 0) / max(64 * d.get("fv_wave_steps", 0), 1),
        "fv_cycles_per_wave_step": d.get("fv_cyc_steps", 0) / max(d.get("fv_wave_steps", 0), 1),
        "fv_steps_frac": d.get("fv_cyc_steps", 0) / max(d.get("fv_cyc_total", 0), 1),
        "fv_wave_steps_per_round": d.get("fv_wave_steps", 0) / max(d.get("fv_rounds", 0), 1),
        "fv_cycles_per_wave": d.get("fv_cyc_total", 0) / max(d.get("fv_waves", 0), 1),
        "uh_cycles_per_unit": {k: d.get(k, 0) / max(d.get("uh_units", 0), 1)
                               for k in ("uh_cyc", "uh_cyc_pro", "uh_cyc_lens", "uh_cyc_lit", "uh_cyc_rest")},
        # expand2 flush: 256-entry wave pieces holding a history marker (the emit's real work)
        "x_marked_piece_frac": d.get("x_pieces_marked", 0) / max(d.get("x_pieces", 0), 1),
        "x_marked_tail_frac": d.get("x_pieces_marked_tail", 0) / max(d.get("x_pieces_marked", 0), 1),
        "x_marker_entry_frac": d.get("x_markers", 0) / max(256 * d.get("x_pieces", 0), 1),
    }
    out = {"raw": d, "derived": derived}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
