#!/bin/bash
# PMC passes: igemm f16x3 in_proj (igf3 case 0), down conv (igf3 case 5) and the halo 3x3 conv (f3 case 0).
MODES=igf3 bash tools/pmc_two.sh "0 5" && MODES=f3 bash tools/pmc_two.sh "0"
