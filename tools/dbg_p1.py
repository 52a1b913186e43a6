import sys, time
sys.path.insert(0, '.')
import numpy as np
from oracle import oracle as O
from tests.rxpkg import rx, synth
for nx, ny, P in [(100, 40, 1), (200, 80, 1), (100, 40, 2)]:
    mesh, st, mech, kw = synth.jet_case(nx, ny, n_species=7, n_part=P)
    om = O.Mechanism(mech)
    cfg = dict(cfl=5.0, max_delta_time=1e6, prandtl_lam=0.72, prandtl_turb=kw['prandtl_turb'], lewis_turb=kw['lewis_turb'],
               mach_inf=kw['mach_inf'], c_mu=kw['c_mu'], pasr_lb=kw['pasr_lb'], lin_tol=1e-6, lin_iter=5, relaxation=1.0)
    N = len(st['V'])
    rp, col = O.bsr_pattern(N, mesh['edges'])
    U, info = O.implicit_step(om, 2, 7, mesh, st, cfg, pattern=(rp, col), part_ptr=mesh['part_ptr'])
    A, b = info['jac'], info['rhs'].ravel()
    pp = mesh['part_ptr']
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), rx.default_cfg(implicit=1, lin_prec=1, **kw))
    s.set_state(st)
    s.Preprocessing_zero(); s.Upwind_Residual(); s.sync(); s.download('RES')
    s.upload('JAC', A); s.upload('RHS', b)
    s.ilu0_build(); s.sync()
    F = O.ilu_build(rp, col, A, part_ptr=pp)
    G = s.download('ILU').reshape(F.shape)
    bad = np.nonzero(~np.isclose(G, F, rtol=1e-12, atol=0).all(axis=(1, 2)))[0]
    rows = np.repeat(np.arange(N), np.diff(rp))
    print(nx, ny, P, 'factor mismatched blocks', len(bad), 'first rows', rows[bad][:10], 'nan', np.isnan(G).sum())
    s.ilu0_apply('RHS', 'SOL'); s.sync()
    x = s.download('SOL'); xr = O.ilu_apply(rp, col, F, b, part_ptr=pp).ravel()
    print('   apply max rel', np.max(np.abs(x - xr)) / np.abs(xr).max(), 'nan', np.isnan(x).sum())
    s.upload('ILU', F)
    s.ilu0_apply('RHS', 'SOL'); s.sync()
    x = s.download('SOL')
    print('   apply(oracle F) max rel', np.max(np.abs(x - xr)) / np.abs(xr).max())
    s.close()
