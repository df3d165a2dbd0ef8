#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a tools/gpu_pmc.sh run: HBM bytes per
launch per kernel = FETCH_SIZE x 2 (gfx950 reports half of wide streaming
reads, MI355X_MICROARCH.md 'HBM') + WRITE_SIZE, both KiB -> bytes.
Also profiles/pmc_valu.json: SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_WAVES per
launch (wave-instructions) per kernel, for bench.py's roofline_valu block.
usage: pmc_traffic.py PMC_DIR TRAFFIC_JSON [VALU_JSON FRAMES_PER_LAUNCH SOURCE]"""
import json
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
pmc = json.loads(subprocess.check_output([sys.executable, "tools/pmc_summary.py", src]))
names = {"k_lpc_analyze": "lpc_analyze", "k_subframe_search": "subframe_search",
         # the 16-bit search and the general kernel's hand-over list run in
         # the same step slot: their per-launch figures add up
         "k_frame_search_ms": "subframe_search", "k_subframe_search16": "subframe_search",
         "k_subframe_search_list": "subframe_search",
         "k_frame_decide": "frame_decide", "k_track_scan": "track_scan",
         "k_frame_pack": "frame_pack", "k_track_md5": "track_md5", "k_track_md5_pair": "track_md5",
         "k_track_md5_roll": "track_md5",
         "k_stream_header": "stream_header",
         # decoder (flac_decode.hip, md5.hip)
         "k_dec_scan": "dec_scan", "k_dec_sync": "dec_scan", "k_dec_hdr": "dec_scan",
         "k_dec_parse": "dec_parse", "k_dec_crc": "dec_parse", "k_dec_spec": "dec_parse", "k_dec_chain": "dec_chain",
         "k_dec_subframe": "dec_subframe", "k_dec_emit": "dec_emit",
         "k_bytes_md5": "dec_md5", "k_bytes_md5_pair": "dec_md5", "k_bytes_md5_roll": "dec_md5",
         "k_pcm_bps": "pcm_bps",
         # resampler (resample.hip)
         "k_rs_phase": "rs_filter", "k_rs_filter": "rs_filter_deep"}
out = {}
for k, v in pmc.items():
    base = k.split("<")[0]
    if base in names and "HBM_read_bytes" in v and "HBM_write_bytes" in v:
        # k_dec_chain runs twice per step (count + write passes): per step
        out[names[base]] = out.get(names[base], 0) + int(v["HBM_read_bytes"] + v["HBM_write_bytes"])
json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1, sort_keys=True))
if len(sys.argv) > 3:
    valu = {}
    for k, v in pmc.items():
        base = k.split("<")[0]
        if base in names and "SQ_INSTS_VALU" in v:
            e = valu.setdefault(names[base], {})
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_INSTS_LDS",
                      "SQ_INSTS_VMEM"):
                if c in v:
                    e[c] = e.get(c, 0) + v[c]
            e["frames"] = int(sys.argv[4])
            e["source"] = sys.argv[5] if len(sys.argv) > 5 else src
    json.dump(valu, open(sys.argv[3], "w"), indent=1, sort_keys=True)
