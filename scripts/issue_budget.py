"""Issue budget of the headline K-step kernel from its gfx950 ISA.

    python scripts/issue_budget.py [--kernel NAME_SUBSTRING] [--json OUT]

Compiles csrc/optimize_lr_persist.hip to assembly (the product flags of
custom_envs_amd/build.py), cuts out the benchmark instance
(optimize_lr_persist_ws_kernel<3,4,false>), finds the row waves' and the
epilogue waves' step loops (the two loops that hold an s_barrier), and counts
per step, by issue class: f64 MFMA, f64 VALU, 32-bit VALU, LDS, VMEM, SALU,
s_waitcnt and s_nop.  The row loop has two bodies behind the clamp-free test
(CE_LR_NOCLAMP); the bounded body is the one that runs on the benchmark data
and is counted (the clamped body and the tie re-walk are listed apart).

The per-class costs ("Issue budget") turn the counts into
time: they are measured, not assumed (profiles/r06_mfma_overlap.jsonl and
profiles/archive/r01_f64_costs.jsonl).
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'custom_envs_amd', 'csrc', 'optimize_lr_persist.hip')


def compile_asm(defines=()):
    out = os.path.join(tempfile.mkdtemp(), 'lp.s')
    cmd = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-x', 'hip', '-O3', '-std=c++17',
           '-I', os.path.join(ROOT, 'include'), '-mllvm', '-amdgpu-mfma-vgpr-form=1',
           '--offload-device-only', '-S', SRC, '-o', out] + ['-D' + d for d in defines]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return open(out).read().split('\n')


def kernel_body(lines, name):
    starts = [i for i, l in enumerate(lines) if l.startswith('_Z') and l.split()[0].endswith(':')
              and name in l]
    if not starts:
        raise SystemExit('kernel %s not found' % name)
    s = starts[0]
    e = next(i for i in range(s, len(lines)) if lines[i].strip().startswith('s_endpgm'))
    return lines[s:e + 1]


def classify(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_', 'flat_', 'scratch_')):
        return 'vmem'
    if op.startswith('s_waitcnt'):
        return 'waitcnt'
    if op.startswith('s_nop'):
        return 'nop'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('v_'):
        return 'valu64' if 'f64' in op else 'valu32'
    return 'other'


def count(body, a, b):
    c, ops = collections.Counter(), collections.Counter()
    for line in body[a:b]:
        t = line.strip()
        if not t or t.startswith(('.', ';')) or t.endswith(':'):
            continue
        op = t.split()[0]
        c[classify(op)] += 1
        ops[op] += 1
    return dict(c), dict(ops.most_common())


def loops(body):
    """(header index, back-branch index) of every loop: a label whose name a
    later branch targets."""
    labels = {l.split()[0][:-1]: i for i, l in enumerate(body) if re.match(r'^\.LBB\w+:', l.strip())}
    out = []
    for i, l in enumerate(body):
        m = re.match(r'\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            out.append((labels[m.group(1)], i))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kernel', default='optimize_lr_persist_ws_kernelILi3ELi4ELb0E')
    ap.add_argument('--define', action='append', default=[])
    ap.add_argument('--json')
    args = ap.parse_args()
    body = kernel_body(compile_asm(args.define), args.kernel)
    # the step loops: outermost loops containing an s_barrier
    cand = []
    for h, b in loops(body):
        if any('s_barrier' in body[i] for i in range(h, b + 1)):
            cand.append((h, b))
    outer = [x for x in cand if not any(y != x and y[0] <= x[0] and x[1] <= y[1] for y in cand)]
    outer.sort()
    res = {'kernel': args.kernel, 'loops': []}
    for h, b in outer:
        whole, ops = count(body, h, b + 1)
        res['loops'].append({'lines': [h, b], 'per_step': whole, 'ops': ops})
    # the row loop: the one with MFMAs; split its two row bodies (the blocks
    # with 28 MFMAs each) from the rest
    for lp in res['loops']:
        lp['role'] = 'row' if lp['per_step'].get('mfma', 0) else 'epilogue'
    row = next((lp for lp in res['loops'] if lp['role'] == 'row'), None)
    if row:
        h, b = row['lines']
        blocks, cur = [], None
        for i in range(h, b + 1):
            if re.match(r'^\.LBB\w+:', body[i].strip()):
                if cur:
                    blocks.append(cur)
                cur = [i, i]
            elif cur:
                cur[1] = i
        if cur:
            blocks.append(cur)
        info = [(blk, count(body, blk[0], blk[1] + 1)[0]) for blk in blocks]
        mf = [(blk, c) for blk, c in info if c.get('mfma', 0) >= 20]
        # the bounded body: the heavy block with fewer f64 VALU (no clamp)
        mf.sort(key=lambda x: x[1].get('valu64', 0))
        if mf:
            bounded = mf[0]
            # the hot path: the blocks ahead of the first row body and the
            # blocks after the last block with an MFMA (the tie re-walk,
            # never taken on the benchmark data, sits between)
            first = min(i for i, (blk, c) in enumerate(info) if c.get('mfma', 0) >= 20)
            last = max(i for i, (blk, c) in enumerate(info) if c.get('mfma', 0) > 0)
            rest = collections.Counter()
            for blk, c in info[:first] + info[last + 1:]:
                rest.update(c)
            total = collections.Counter(bounded[1])
            total.update(rest)
            row['bounded_body'] = bounded[1]
            row['outside_bodies'] = dict(rest)
            row['per_step_bounded'] = dict(total)
    txt = json.dumps(res, indent=1)
    if args.json:
        with open(args.json, 'w') as fh:
            fh.write(txt)
    for lp in res['loops']:
        print(lp['role'], 'per step:', lp.get('per_step_bounded', lp['per_step']))
        if 'bounded_body' in lp:
            print('   bounded row body:', lp['bounded_body'])
            print('   around it       :', lp['outside_bodies'])
    return 0


if __name__ == '__main__':
    sys.exit(main())
