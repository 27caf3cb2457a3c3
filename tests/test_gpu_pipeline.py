"""The Riccati solve as a launch pipeline (iterations with hand-off -> lock-step polish -> single
kernel for the rejected polishes; batches of 49,152 instances and more) against the same solve in
ONE kernel.  carmpc_solve_batch_noalloc always runs the single kernel (it brings its own claim
counter), so the two entry points give the two paths on identical inputs: statuses and iteration
counts must be equal, u to 1e-12 (both paths run the same arithmetic per instance; the pipeline
only changes which launch performs which part)."""
import ctypes

import numpy as np
import pytest

from conftest import TERMINAL_SETS
from test_zz_no_alloc import _call, _x0

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("env,N", [("RoadMultipleCarsEnv", 20), ("RoadEnv", 20), ("RoadOneCarEnv", 10), ("RoadEnv", 15),
                                   ("RoadMultipleCarsEnv", 25), ("RoadOneCarEnv", 5)])
def test_pipeline_equals_single_kernel(gpu_available, env, N):
    import torch
    from oracle import assembly as oa
    from carmpc_amd import _native
    from carmpc_amd.qp import QPProblem, SolverSettings
    lib = _native.load()
    asm = oa.build(env, N, terminal_set_dir=TERMINAL_SETS)
    qp = QPProblem(N=N, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    assert qp.kernel == 7
    B = 65536
    x = _x0(np.random.default_rng(11), asm.goal[0], B)
    x[:, 0] = asm.goal[0] - (asm.goal[0] - x[:, 0]) * min(1.0, N / 20 * 1.05)      # (reachable within the horizon)
    X = torch.as_tensor(x).to(qp.device)
    settings = SolverSettings()
    u1, st1, it1 = _call(lib.carmpc_solve_batch, qp, X, settings)            # pipeline
    u0, st0, it0 = _call(lib.carmpc_solve_batch_noalloc, qp, X, settings)    # single kernel
    torch.cuda.synchronize()
    assert int((st1 < 0).sum()) == 0                                         # every instance got a result
    assert torch.equal(st1, st0) and torch.equal(it1, it0)
    ok = (st0 == 0).cpu().numpy()
    assert ok.sum() > B // 8
    np.testing.assert_allclose(u1.cpu().numpy()[ok], u0.cpu().numpy()[ok], rtol=0, atol=1e-12)
    assert torch.equal(u1[st1 != 0], u0[st1 != 0])                           # (infeasible instances: last iterate or zeros)


def test_pipeline_with_disturbance_and_xref_equals_chunked_single_kernel(gpu_available):
    """Per-instance disturbance estimates and explicit references through the pipeline (65,536
    instances in one call) against the same instances solved in chunks below the pipeline's
    size threshold (single kernel)."""
    import torch
    from oracle import assembly as oa
    from carmpc_amd.qp import QPProblem
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    qp = QPProblem(N=20, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    qp.set_disturbance(np.array([0.0, 0.0, 0.02, 0.05]))
    B, chunk = 65536, 16384
    rng = np.random.default_rng(5)
    X = torch.as_tensor(_x0(rng, asm.goal[0], B)).to(qp.device)
    D = torch.as_tensor(rng.uniform(-0.5, 0.5, B)).to(qp.device)
    R = torch.as_tensor(np.tile(asm.goal, (B, 1)) + rng.normal(scale=0.05, size=(B, 4))).to(qp.device)
    u1, st1, it1 = qp.solve(X, xref=R, dist=D)
    parts = [qp.solve(X[i:i + chunk], xref=R[i:i + chunk], dist=D[i:i + chunk]) for i in range(0, B, chunk)]
    torch.cuda.synchronize()
    u0 = torch.cat([p[0] for p in parts]); st0 = torch.cat([p[1] for p in parts]); it0 = torch.cat([p[2] for p in parts])
    assert torch.equal(st1, st0) and torch.equal(it1, it0)
    assert int((st0 == 0).sum()) > B // 8
    assert torch.equal(u1, u0)


def test_short_horizon_layouts_agree(gpu_available):
    """N = 10 problems whose rows fit one slot segment run four QPs per wavefront from 16,384 instances on and
    two per wavefront below: a batch solved whole (pipeline, four per wave), in chunks of 20,000 (single kernel,
    four per wave) and in chunks of 4,000 (single kernel, two per wave) gives the same statuses and iteration
    counts, and u to 1e-12 (the layouts order their sums differently)."""
    import torch
    from oracle import assembly as oa
    from carmpc_amd.qp import QPProblem
    asm = oa.build("RoadMultipleCarsEnv", 10, terminal_set_dir=TERMINAL_SETS)
    qp = QPProblem(N=10, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    B = 60000
    x = _x0(np.random.default_rng(17), asm.goal[0], B)
    x[:, 0] = asm.goal[0] - (asm.goal[0] - x[:, 0]) * 0.5
    X = torch.as_tensor(x).to(qp.device)
    u0, s0, i0 = qp.solve(X)
    torch.cuda.synchronize()
    assert int((s0 == 0).sum()) > B // 8
    for chunk in (20000, 4000):
        parts = [qp.solve(X[i:i + chunk]) for i in range(0, B, chunk)]
        torch.cuda.synchronize()
        u1 = torch.cat([p[0] for p in parts]); s1 = torch.cat([p[1] for p in parts]); i1 = torch.cat([p[2] for p in parts])
        assert torch.equal(s1, s0), chunk
        same = float((i1 == i0).double().mean())
        assert same >= 0.999 and int((i1 - i0).abs().max()) <= 2, (chunk, same)
        ok = (s0 == 0)
        assert float((u1[ok] - u0[ok]).abs().max()) <= 1e-9, chunk


def test_call_larger_than_the_saved_iterates(gpu_available):
    """The iteration launch saves the iterate of every hand-off so that a rejected polish resumes from it, in
    memory bounded per call (carmpc_internal.h: kRicStateMaxBytes, 279,620 instances).  A call beyond that
    bound mixes the three kinds of work in its final launch -- resumed retries, retries that start over, and
    the fresh instances it takes from the end of the batch when some retries start over -- and must return
    what calls below the bound return (every retry resumed, no fresh instances): statuses, iteration counts
    and u bit for bit, since every path runs the same arithmetic per instance."""
    import torch
    from oracle import assembly as oa
    from carmpc_amd.qp import QPProblem
    asm = oa.build("RoadEnv", 20, terminal_set_dir=TERMINAL_SETS)     # (mostly feasible: more hand-offs than the bound holds)
    qp = QPProblem(N=20, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    B, part = 393216, 131072
    x = _x0(np.random.default_rng(23), asm.goal[0], B)
    X = torch.as_tensor(x).to(qp.device)
    u1, st1, it1 = qp.solve(X)
    torch.cuda.synchronize()
    assert int((st1 == 0).sum()) > 300000
    for k in range(0, B, part):
        u0, st0, it0 = qp.solve(X[k:k + part])
        torch.cuda.synchronize()
        bad = ((st0 != st1[k:k + part]) | (it0 != it1[k:k + part])).nonzero().flatten()
        assert bad.numel() == 0, (k, bad[:8].tolist(), st0[bad[:8]].tolist(), st1[k:k + part][bad[:8]].tolist())
        assert torch.equal(u0, u1[k:k + part])


def test_work_memory_is_reused_between_calls(gpu_available):
    """The pipeline's work memory (lists and saved iterates, about 1 GB for 131,072 instances) comes from a
    stream-ordered pool that keeps it between calls: after a warm call, synchronised calls of the same size leave
    the free device memory where it was (no growth per call, no allocation and release per call)."""
    import torch
    from oracle import assembly as oa
    from carmpc_amd.qp import QPProblem
    asm = oa.build("RoadOneCarEnv", 20, terminal_set_dir=TERMINAL_SETS)
    qp = QPProblem(N=20, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    B = 131072
    X = torch.as_tensor(_x0(np.random.default_rng(3), asm.goal[0], B)).to(qp.device)
    out = (torch.empty((B, qp.n), dtype=torch.float64, device=qp.device),
           torch.empty(B, dtype=torch.int32, device=qp.device), torch.empty(B, dtype=torch.int32, device=qp.device))
    for _ in range(2):
        qp.solve(X, out=out)
        torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    st0 = out[1].clone()
    for _ in range(10):
        qp.solve(X, out=out)
        torch.cuda.synchronize()
        assert torch.cuda.mem_get_info()[0] == free0
    assert torch.equal(out[1], st0)


@pytest.mark.parametrize("N", [10, 20])
def test_paired_rows_through_the_pipeline(gpu_available, tmp_path, N):
    """Problems whose terminal set is the goal box (missing terminal-set file, mpc.py:107-117: opposite rows
    paired into equalities, which the polish acceptance test handles through a shared scratch buffer) at a
    batch size that runs as three launches -- with four QPs per wavefront at N = 10 and two at N = 20:
    statuses and iteration counts of every instance against the C oracle."""
    import torch
    from oracle import assembly as oa
    from oracle.cpu import CpuProblem
    from carmpc_amd.qp import QPProblem
    asm = oa.build("RoadEnv", N, terminal_set_dir=str(tmp_path))
    assert asm.term_file is None
    qp = QPProblem(N=N, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    assert qp.kernel == 7
    B = 65536
    rng = np.random.default_rng(100 + N)
    X = np.stack([rng.uniform(30 - 0.2 * N, 30, B), rng.uniform(1, 2, B), rng.uniform(-0.05, 0.05, B),
                  rng.uniform(-0.2, 0.2, B)], axis=1)
    uc, sc, ic = CpuProblem(asm).solve(X)
    assert int((sc == 0).sum()) > B // 4
    Xd = torch.as_tensor(X).cuda()
    for _ in range(3):
        u, st, it = qp.solve(Xd)
        torch.cuda.synchronize()
        st, it = st.cpu().numpy(), it.cpu().numpy()
        np.testing.assert_array_equal(st, sc)
        ok = sc == 0
        np.testing.assert_array_equal(it[ok], ic[ok])
        assert np.abs(u.cpu().numpy()[ok] - uc[ok]).max() <= 1e-6
