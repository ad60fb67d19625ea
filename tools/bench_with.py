"""Run bench.py with a process-wide kernel-form selector applied first (A/B runs):
    python tools/bench_with.py --proj-tile 128 -- --steps 60 --no-roofline"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    rest = argv[argv.index('--') + 1:] if '--' in argv else []
    opts = argv[:argv.index('--')] if '--' in argv else argv
    from weatherconverter_amd import kernels as K
    for i in range(0, len(opts), 2):
        if opts[i] == '--proj-tile':
            K.set_proj_tile(int(opts[i + 1]))
        else:
            raise SystemExit(f'unknown option {opts[i]}')
    sys.argv = [os.path.join(ROOT, 'bench.py')] + rest
    runpy.run_path(sys.argv[0], run_name='__main__')


if __name__ == '__main__':
    main()
