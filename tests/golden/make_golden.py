"""Generate tests/golden/ref_fixtures.npz from the REAL reference (flang-built oracle/_ref).

Run in the build container only (needs /root/reference and flang):
    make -C oracle ref && python tests/golden/make_golden.py

Inputs are produced here with a seeded numpy RNG and stored explicitly next to the outputs (the
reference's own tests draw from the unseeded, compiler-specific `random_number`),
using the same recipes as the reference tests:
  * tridiagonal systems: tests/tridiag/test_tdma_utils.f90:12-67 (U[0,1) a, b, c, x; diagonal
    multiplied by 10 until |b| >= |a| + |c|; a(1) = c(n) = 0 unless periodic; d = A x)
  * 1-D compact fields: sin on a 2*pi periodic line (tests/grad/test_grad_1d.f90:89-96) + random
  * 3-D compact fields: random and sum-of-sines (tests/lapl/test_lapl.f90:87-100)
  * 7-point operator fields: random on periodic grids with uniform and non-uniform spacing
    (src/poissbox.f90:128-148 evaluate_laplacian_pointwise + src/coefficients.f90:22-48, cut out
    of those PETSc-dependent files by oracle/Makefile)
The Fortran program oracle/_ref/gen_fixtures evaluates the reference routines on these inputs.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
GEN = os.path.join(REPO, "oracle", "_ref", "gen_fixtures")


def tdma_system(rng, n, periodic):
    a, b, c, x = (rng.random(n) for _ in range(4))
    if not periodic:
        a[0] = 0.0
        c[n - 1] = 0.0
    for i in range(n):
        while b[i] == 0.0:
            b[i] = rng.random()
        while abs(b[i]) < abs(a[i]) + abs(c[i]):
            b[i] = 10 * b[i]
    d = np.empty(n)
    d[0] = b[0] * x[0] + c[0] * x[1]
    if periodic:
        d[0] = a[0] * x[n - 1] + d[0]
    for i in range(1, n - 1):
        d[i] = a[i] * x[i - 1] + b[i] * x[i] + c[i] * x[i + 1]
    d[n - 1] = a[n - 1] * x[n - 2] + b[n - 1] * x[n - 1]
    if periodic:
        d[n - 1] = c[n - 1] * x[0] + d[n - 1]
    return a, b, c, x, d


def sines3(n, h, shift):
    """f(i,j,k) = sin(x)+sin(y)+sin(z) at (i+shift)*h, Fortran order flattened."""
    x = (np.arange(n[0]) + shift) * h[0]
    y = (np.arange(n[1]) + shift) * h[1]
    z = (np.arange(n[2]) + shift) * h[2]
    f = np.sin(z)[:, None, None] + np.sin(y)[None, :, None] + np.sin(x)[None, None, :]
    return f.reshape(-1)


def main():
    if not os.path.exists(GEN):
        sys.exit("build the reference first: make -C oracle ref")
    rng = np.random.default_rng(20231015)
    cases = []  # (name, op, n3, h3, input array)

    for n in (128, 7, 512):
        for periodic in (False, True):
            a, b, c, x, d = tdma_system(rng, n, periodic)
            tag = f"n{n}_{'per' if periodic else 'np'}"
            abcd = np.concatenate([a, b, c, d])
            cases.append((f"tdma__{tag}", "tdma", (n, 1, 1), (0, 0, 0), abcd, x))
            cases.append((f"tdma_periodic__{tag}", "tdma_periodic", (n, 1, 1), (0, 0, 0), abcd, x))
            if not periodic:
                cases.append((f"fwd_sweep__{tag}", "fwd_sweep", (n, 1, 1), (0, 0, 0), abcd, x))
                du = b * x
                du[:-1] += c[:-1] * x[1:]
                cases.append((f"bwd_sweep__{tag}", "bwd_sweep", (n, 1, 1), (0, 0, 0),
                              np.concatenate([b, c, du]), x))

    two_pi = 2 * np.pi
    for n in (128, 33, 3, 512):
        dx = two_pi / n
        fsin = np.sin((np.arange(n) + 0.5) * dx)
        frnd = rng.random(n) * 2 - 1
        for tag, f in (("sin", fsin), ("rnd", frnd)):
            for op in ("grad_1d", "div_1d", "interp_1d", "interp_1d_div"):
                cases.append((f"{op}__n{n}_{tag}", op, (n, 1, 1), (dx, 0, 0), f, None))

    for n3 in ((16, 16, 16), (8, 12, 10), (3, 4, 5)):
        h3 = tuple(two_pi / m for m in n3)
        N = int(np.prod(n3))
        f = rng.random(N) * 2 - 1
        v = rng.random(3 * N) * 2 - 1
        tag = "x".join(map(str, n3))
        for op in ("grad", "interp", "interp_div", "lapl"):
            cases.append((f"{op}__{tag}_rnd", op, n3, h3, f, None))
        cases.append((f"div__{tag}_rnd", "div", n3, h3, v, None))
        cases.append((f"lapl__{tag}_sin", "lapl", n3, h3, sines3(n3, h3, 0.5), None))

    # 7-point operator (SURVEY.md §8(c) golden vector 4): the reference's own
    # evaluate_laplacian_pointwise + lapl_star_coeffs on periodic grids, unit-cube and non-uniform
    # spacings (drawn after every case above, so those fixtures are unchanged)
    for n3, L in (((16, 16, 16), (1.0, 1.0, 1.0)), ((17, 12, 9), (1.0, 2.0, 0.5)),
                  ((24, 20, 10), (2.4, 0.74, 2.9)), ((32, 32, 32), (1.0, 1.0, 1.0)),
                  ((9, 7, 5), (3.0, 1.0, 7.0))):
        h3 = tuple(Lq / m for Lq, m in zip(L, n3))
        N = int(np.prod(n3))
        tag = "x".join(map(str, n3))
        cases.append((f"star__{tag}_rnd", "star", n3, h3, rng.random(N) * 2 - 1, None))
        if n3 == (16, 16, 16):
            cases.append((f"star__{tag}_sin", "star", n3, h3, sines3(n3, h3, 0.0), None))

    out = {}
    with tempfile.TemporaryDirectory() as td:
        lines = []
        for idx, (name, op, n3, h3, arr, _) in enumerate(cases):
            fin = os.path.join(td, f"in{idx}.bin")
            fout = os.path.join(td, f"out{idx}.bin")
            arr.astype("<f8").tofile(fin)
            lines.append(f"{op} {n3[0]} {n3[1]} {n3[2]} {h3[0]!r} {h3[1]!r} {h3[2]!r} '{fin}' '{fout}'")
        man = os.path.join(td, "manifest.txt")
        with open(man, "w") as fh:
            fh.write("\n".join(lines) + "\n")
        subprocess.run([GEN, man], check=True)
        for idx, (name, op, n3, h3, arr, xs) in enumerate(cases):
            res = np.fromfile(os.path.join(td, f"out{idx}.bin"), dtype="<f8")
            out[f"{name}__in"] = arr
            out[f"{name}__out"] = res
            out[f"{name}__meta"] = np.array([n3[0], n3[1], n3[2], h3[0], h3[1], h3[2]], dtype=np.float64)
            if xs is not None:
                out[f"{name}__x"] = xs
    dst = os.path.join(HERE, "ref_fixtures.npz")
    np.savez_compressed(dst, **out)
    print(f"wrote {dst}: {len(cases)} cases, {os.path.getsize(dst)} bytes")


if __name__ == "__main__":
    main()
