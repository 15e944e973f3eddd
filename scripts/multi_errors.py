"""Print the worst HIP-vs-oracle differences on the MultiOptLRs fixtures.

Run on the GPU box:  python scripts/multi_errors.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), os.pardir))
from custom_envs_amd.multi_engine import MultiOptEngine  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), os.pardir, 'tests', 'golden')
CASES = [('multi_func2_h5', 'func', 400, 5), ('multi_func4_h5', 'func4', 400, 5),
         ('multi_func4_h3_b25', 'func4', 25, 3)]


def main():
    for name, problem, mb, hist in CASES:
        fx = np.load(os.path.join(GOLDEN, name + '.npz'))
        eng = MultiOptEngine(1, problem, max_batches=mb, max_history=hist)
        eng.reset()
        worst = {'obs_exact': 0, 'theta_exact': 0, 'reward_exact': 0, 'steps': 0}
        info_err = np.zeros(14)
        theta_err = 0.0
        for t in range(fx['actions'].shape[0]):
            out = eng.step(fx['actions'][t].reshape(-1))
            worst['steps'] += 1
            worst['obs_exact'] += int(np.array_equal(out['obs'], fx['obs'][t]))
            worst['reward_exact'] += int(out['reward'][0] == np.float32(fx['reward'][t]))
            if not fx['done'][t]:
                th = eng.get_state()['theta'][0]
                worst['theta_exact'] += int(np.array_equal(th, fx['theta'][t].astype(np.float32)))
                theta_err = max(theta_err, float(np.max(np.abs(th - fx['theta'][t]) /
                                                        np.maximum(np.abs(fx['theta'][t]), 1e-30))))
            ref = fx['info'][t]
            fin = np.isfinite(ref)
            e = np.zeros(14)
            e[fin] = np.abs(out['info'][0][fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-30)
            info_err = np.maximum(info_err, e)
        eng.close()
        print(name, worst, 'theta rel', theta_err)
        print('   info rel', np.array2string(info_err, precision=2))


if __name__ == '__main__':
    main()
