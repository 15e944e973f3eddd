"""The f64 kernels' table exponential (exp_neg_tab) on the
host: the committed table is what scripts/gen_exp2_table.py generates
(2^(j/2048) correctly rounded), and the algorithm restated in C over that
table stays within 1.5 ulp of expl over [-700, 750], with e^0 == 1 exactly
(the full-batch kernels' argmax relies on it)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'custom_envs_amd', 'csrc', 'exp2_table.h')


def test_committed_table_is_the_generated_one(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, 'scripts'))
    import gen_exp2_table
    vals = gen_exp2_table.table()
    text = open(HEADER).read()
    assert all(v.hex() in text for v in vals)
    assert vals[0] == 1.0 and len(vals) == 2048
    assert '#define CE_EXP2_TAB_SIZE 2048' in text


@pytest.mark.skipif(shutil.which('gcc') is None, reason='needs gcc')
def test_table_exp_accuracy(tmp_path):
    exe = str(tmp_path / 'texp')
    subprocess.run(['gcc', '-O2', '-ffp-contract=off', '-I', os.path.dirname(HEADER),
                    os.path.join(ROOT, 'tests', 'exp_table', 'texp.c'), '-o', exe, '-lm'], check=True)
    worst, exact_one = subprocess.run([exe], check=True, capture_output=True,
                                      text=True).stdout.split()
    assert float(worst) <= 1.5, worst
    assert exact_one == '1'
