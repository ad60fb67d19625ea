"""Reconcile bench.py's per-kernel table (roofline.mfma_kernels: per-launch re-issue timings of one
eager forward) with the rocprofv3 trace of the timed graph replays (tools/step_table.py --json).

Usage: python tools/reconcile.py <bench json line file> <step_table.json>
Prints per instantiation: ms per step from the trace, ms per forward from the bench, their ratio,
and the totals over the instantiations both contain (the verdict's bar: within 3 %)."""
import json
import sys


def main():
    line = [ln for ln in open(sys.argv[1]) if ln.startswith('{')][-1]
    bench = json.loads(line)['roofline']['mfma_kernels']
    trace = {k['kernel']: k for k in json.load(open(sys.argv[2]))['kernels']}
    tb = tt = 0.0
    print(f'{"kernel":75s} {"trace ms":>9s} {"bench ms":>9s} {"ratio":>6s}')
    for name, b in sorted(bench.items(), key=lambda kv: -kv[1]['ms']):
        t = trace.get(name)
        tms = t['ms_per_step'] if t else float('nan')
        if t:
            tb += b['ms']
            tt += tms
        print(f'{name[:75]:75s} {tms:9.3f} {b["ms"]:9.3f} {b["ms"] / tms if t else float("nan"):6.3f}')
    print(f'common instantiations: trace {tt:.3f} ms/step, bench {tb:.3f} ms/forward, ratio {tb / tt:.4f}')
    missing = [k for k in bench if k not in trace]
    if missing:
        print('in bench but not in trace:', missing)


if __name__ == '__main__':
    main()
