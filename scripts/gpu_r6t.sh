#!/bin/bash
# round 6 t: texture address / data unit busy cycles + vector-memory
# instruction counts beside the GRBM clock, for the four lines' timed
# configurations (is the gather path, not the VALU, what binds them?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6t}; mkdir -p $O
export PMC_SET="TA_BUSY_avr TD_BUSY_avr SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
export PMC_TAG=ta
D=/tmp/ngt_ta_anng_$$
PMC_LAST=12 bash scripts/pmc_clk.sh $O c2 --eps 0.058203125 --sweep-nq 10000 --pmc-launches 6 --no-cpu --anng-line off \
  --c3-line off --qg-line off || exit 1
PMC_LAST=3 bash scripts/pmc_clk.sh $O anng --graph anng --anng-dir $D --capi-line off --eps 0.1279296875 \
  --sweep-nq 10000 --pmc-launches 3 --no-cpu || exit 1
PMC_LAST=3 bash scripts/pmc_clk.sh $O qg --mode qg --graph anng --anng-dir $D --eps 0.09772 --expansion 3 \
  --sweep-nq 10000 --pmc-launches 3 --no-cpu --anng-line off --c3-line off --qg-line off || exit 1
PMC_LAST=3 bash scripts/pmc_clk.sh $O c3 --config c3 --eps 0.056640625 --sweep-nq 10000 --pmc-launches 3 --no-cpu \
  --anng-line off --c3-line off --qg-line off || exit 1
rm -rf $D
