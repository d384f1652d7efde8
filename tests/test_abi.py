"""The C-ABI library loads, exports exactly what include/nlot.h declares, and the ctypes struct
layouts agree with the C compiler's (checked through the oracle, which includes the same header)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "nlot.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\([^;{]*\)\s*;", src))
    return {n for n in names if n not in {"if", "return", "sizeof"}}


def test_header_lists_all_symbols():
    from nlotrajectories_amd._lib import EXPORTED

    assert header_functions() == set(EXPORTED)


def test_library_exports_every_symbol():
    import ctypes as C

    from nlotrajectories_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    L = C.CDLL(_lib.LIB_PATH)
    for name in header_functions():
        assert hasattr(L, name), name
    ver = int(re.search(r"#define NLOT_ABI_VERSION (\d+)", open(os.path.join(ROOT, "include", "nlot.h")).read())[1])
    assert _lib.lib().nlot_abi_version() == ver


def test_struct_layouts_match_header():
    import ctypes as C

    import oracle as O
    from nlotrajectories_amd import _abi

    L = O.lib()
    assert L.oracle_sizeof_problem() == C.sizeof(_abi.NlotProblem)
    assert L.oracle_sizeof_options() == C.sizeof(_abi.NlotSolverOptions)
    assert L.oracle_sizeof_mlpdesc() == C.sizeof(_abi.NlotMlpDesc)
    assert L.oracle_sizeof_stats() == C.sizeof(_abi.NlotSolveStats)


def test_default_options_agree():
    import ctypes as C

    from nlotrajectories_amd import _abi, _lib

    o = _abi.NlotSolverOptions()
    _lib.lib().nlot_default_options(C.byref(o))
    d = _abi.default_options()
    for k, _ in o._fields_:
        assert getattr(o, k) == getattr(d, k), k


def test_workspace_holds_the_slots_only():
    """ABI v10: the solver's state is slot-indexed, so B instances streamed through S slots need the workspace of S
    (plus nothing per instance: outputs go to the caller's arrays when an instance finishes)."""
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.solver import workspace_bytes

    full = workspace_bytes(METRIC_PROBLEM, 4096)
    assert workspace_bytes(METRIC_PROBLEM, 4096, 0) == full
    assert workspace_bytes(METRIC_PROBLEM, 4096, 4096) == full
    assert workspace_bytes(METRIC_PROBLEM, 1 << 20, 4096) == full
    assert workspace_bytes(METRIC_PROBLEM, 4096, 512) == workspace_bytes(METRIC_PROBLEM, 512) < full


def test_solve_batch_refuses_bad_arguments_before_the_device():
    """nlot_solve_batch validates on the host and fails loudly (NLOT_ERR_INVALID + nlot_last_error) before any device
    call, so these run without a GPU: an empty or oversized batch, a general_bounds value other than 0 / 1, an unknown
    mu_strategy, a learned-SDF problem without a net, null output pointers."""
    import ctypes as C

    from nlotrajectories_amd import _abi, _lib
    from nlotrajectories_amd.problem import BENCHMARKS, METRIC_PROBLEM

    L = _lib.lib()
    pc = BENCHMARKS["b2"]["problem"].to_c()

    def call(opt, B, prob=pc):
        rc = L.nlot_solve_batch(C.byref(prob), C.byref(opt), None, None, None, None, None, None, None, None, None,
                                None, B, None, 0, None)
        return rc, L.nlot_last_error().decode()

    base = _abi.gpu_options()
    assert call(base, 0) == (-1, "B out of range")
    assert call(base, (1 << 26) + 1) == (-1, "B out of range")
    rc, msg = call(base, 4)
    assert rc == -1 and msg == "nlot_solve_batch: null pointer"
    assert base.general_bounds == 1  # the reference's NLP form (runner.py:67-69,101-103) is the default
    o = _abi.gpu_options()
    o.general_bounds = 2
    rc, msg = call(o, 4)
    assert rc == -1 and "general_bounds" in msg
    o = _abi.gpu_options()
    o.mu_strategy = 2
    assert call(o, 4)[0] == -1 and "mu_strategy" in call(o, 4)[1]
    rc, msg = call(base, 4, METRIC_PROBLEM.to_c())
    assert rc == -1 and "requires an NlotMlp" in msg
