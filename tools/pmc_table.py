"""Per-kernel PMC summary from rocprofv3 --pmc CSVs: mean counter value per dispatch of each conv /
attention kernel, merged over passes.  Usage: python tools/pmc_table.py gpurun_out/pmc_igf3_c0_p1 gpurun_out/pmc_igf3_c0_p2"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            per = defaultdict(float)
            names = {}
            for r in csv.DictReader(open(f)):
                k = (r['Dispatch_Id'], r['Counter_Name'])
                per[k] += float(r['Counter_Value'])
                names[r['Dispatch_Id']] = r['Kernel_Name']
            for (disp, cn), v in per.items():
                acc[names[disp]][cn].append(v)
    return acc


def main():
    acc = load(sys.argv[1:])
    for kern, cs in acc.items():
        if 'conv' not in kern and 'attention' not in kern and 'attn' not in kern:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(kern[:100])
        for c in sorted(m):
            print(f'  {c:28s} {m[c]:16.4g}')
        busy = m.get('SQ_BUSY_CYCLES') or m.get('GRBM_GUI_ACTIVE')
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in m and 'GRBM_GUI_ACTIVE' in m:
            # MFMA busy per SIMD: the counter sums 1024 SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs
            print(f'  MFMA busy fraction ~ {m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024):.3f}')
        if 'SQ_WAIT_INST_ANY' in m and 'SQ_WAVE_CYCLES' in m:
            print(f'  wait_inst_any / wave_cycles = {m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]:.3f}, '
                  f'wait_any / wave_cycles = {m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]:.3f}')


if __name__ == '__main__':
    main()
