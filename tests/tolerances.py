"""Parity bounds of the GPU tests per engine precision, engine vs the fp64 oracle on identical inputs.

fp64 engine (GCS_PRECISION_F64, the default; the reference's own arithmetic): the bounds leave room only for a
different summation order of the pair forces, fused multiply-adds and last-ulp differences of the device libm
(sqrt, log, sincospi) -- measured differences are ~1e-13 and below.  fp32 engine (GCS_PRECISION_F32): fp32 rounding
of positions and forces.  Integer / index results (pair sets, contact counts, quantised samples) are bit-exact at
both precisions and are asserted with array_equal.
"""
import numpy as np
import pytest

PRECISIONS = (64, 32)
X = {64: 1e-9, 32: 2e-5}            # positions, max |dx| after <= 60 steps with identical noise
F_REL = {64: 1e-10, 32: 1e-4}       # forces: max |dF| <= F_REL * max |F| + F_ABS
F_ABS = {64: 1e-10, 32: 1e-3}
E_REL = {64: 1e-10, 32: 1e-5}       # energies (relative; per kind with E_ABS absolute for kinds near zero)
E_ABS = {64: 1e-9, 32: 1e-4}
WALL_REL = {64: 1e-12, 32: 1e-7}    # wall semiaxes after a run
REACT = {64: (1e-9, 1e-9), 32: (1e-3, 1e-2)}  # wall reactions (rtol, atol) after a run
REACT_FORCES = {64: (1e-10, 1e-10), 32: (1e-4, 1e-3)}  # wall reactions of one force evaluation

precisions = pytest.mark.parametrize("prec", PRECISIONS)


def assert_forces_close(fe, fo, prec):
    scale = np.abs(fo).max()
    err = np.abs(fe - fo).max()
    assert err <= F_REL[prec] * scale + F_ABS[prec], (prec, err, scale)


def assert_positions_close(xe, xo, prec):
    err = np.abs(xe - xo).max()
    assert err <= X[prec], (prec, err)
