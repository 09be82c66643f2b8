#!/bin/bash
# Round-6 profile summaries from gpurun_out/prof/r06_c{2,3,4,5} (tools/gpu_prof.sh r06 ...): kernel stats,
# per-kernel PMC bytes and the bench's traffic files (profiles/pmc_traffic*.json)
set -e
cd "$(dirname "$0")/.."
python3 tools/pmc_summary.py r06_c2 stencil_plain_kernel 100000000 r06_c2 c2
python3 tools/pmc_summary.py r06_c3 kcep_runs_sim,runs_chunk_scan,runs_results,runs_emit 10000000 r06_c3 c3
python3 tools/pmc_summary.py r06_c4 kcep_nfa_wave,kcep_nfa_order,nfa_order_count,nfa_order_place,seg_count,scan_sums_reg,seg_write,set_words,scan_blocks,scan_sums_pair,scan_final,nfa_compact_matches,nfa_compact_entries,gather_words 1200000 r06_c4 c4
python3 tools/pmc_summary.py r06_c5 stencil_kernel 1000000000 r06_c5 c5
