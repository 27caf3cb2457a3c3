"""Re-pin the oracle iteration counts stored in tests/golden/qp_*.npz after an algorithm change
(here POLISH_MU 1e-8 -> 1e-6): statuses and u* must be unchanged (asserted), only `iters` is
rewritten.  x0, status, u_star and margin stay as tools/make_golden.py wrote them."""
import os
import sys

import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import assembly as oa, qp as oq
G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden')
for name, N in [("RoadEnv", 10), ("RoadEnv", 20), ("RoadOneCarEnv", 20), ("RoadMultipleCarsEnv", 20)]:
    f = os.path.join(G, f"qp_{name}_N{N}.npz")
    g = dict(np.load(f))
    asm = oa.build(name, N, terminal_set_dir=os.path.join(os.path.dirname(G), '..', 'terminal_sets'))
    new_it = []
    for i, x in enumerate(g['x0']):
        r = oq.solve_instance(asm, x)
        assert r['status'] == g['status'][i], (name, i)
        if r['status'] == 0:
            assert np.abs(r['u'] - g['u_star'][i]).max() <= 1e-8, (name, i)
        new_it.append(r['iters'])
    new_it = np.array(new_it, np.int32)
    ok = g['status'] == 0
    print(name, N, 'iters mean old %.2f new %.2f' % (g['iters'][ok].mean(), new_it[ok].mean()))
    g['iters'] = new_it
    np.savez(f, **g)
