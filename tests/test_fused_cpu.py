"""K18 expression compiler (CPU side): which trees become one fused kernel and which stay on the operator path
(the kernel itself is checked against the operator path in tests/test_kernels_gpu.py)."""
import numpy as np
import pytest
import pandas as pd


def test_fused_compiler_coverage(spark):
    from cdnaml.models.util import local_batch
    from cdnaml.sql import fused
    from cdnaml.sql import functions as F
    df = spark.createDataFrame(pd.DataFrame({"x": np.arange(10.0), "y": np.arange(10.0).astype(np.float32),
                                             "k": np.arange(10).astype(np.int32), "s": list("abcdefghij")}))
    b = local_batch(df, ["x", "y", "k", "s"])
    x, y, k, s = F.col("x"), F.col("y"), F.col("k"), F.col("s")
    fusable = [x * 2.0 + 1.0, F.log(x + 1.0) - F.exp(x * 0.1), (x > 1) & (k < 3), F.when(x > 2, x * 2.0).otherwise(0.0),
               (x * 3.0).cast("int") + 0.5, F.round(x / 3.0, 2) * 2.0, F.isnull(x * 1.0) | F.isnan(x / 2.0),
               y * 1.0 + k, F.sqrt(F.abs(x - 5.0)) * 2.0]
    for e in fusable:
        assert fused.can_fuse(e._expr, b), str(e._expr)
    not_fusable = [x + 1.0,                       # a single operator: already one kernel
                   y.cast("float") * y.cast("float") + 1.0,   # float32 arithmetic rounds per op
                   k * k + k,                     # integer arithmetic (overflow semantics)
                   F.lower(s),                    # strings stay on the dictionary path
                   F.when(s == "a", x * 2.0).otherwise(1.0) + x]
    for e in not_fusable:
        assert not fused.can_fuse(e._expr, b), str(e._expr)


def test_fused_programs_match_operator_path_on_host(spark):
    """Every compiled program, run through the host reference of the kernel's semantics (fused.interpret), equals
    the operator path on data with nulls, NaN, zero divisors and out-of-domain logs."""
    from cdnaml.models.util import local_batch
    from cdnaml.sql import fused
    from cdnaml.sql import functions as F
    from cdnaml.sql.column import EvalContext
    rng = np.random.default_rng(3)
    n = 3001
    x = rng.normal(size=n) * 5
    x[::17] = 0.0
    x[::29] = np.nan
    pdf = pd.DataFrame({"x": x, "y": rng.normal(size=n).astype(np.float32), "k": rng.integers(-3, 4, n).astype(np.int32),
                        "big": rng.integers(0, 10 ** 6, n)})
    pdf["b"] = pdf.k > 0
    pdf.loc[::13, "x"] = None
    pdf["k"] = pdf["k"].astype("Int32")
    pdf.loc[::11, "k"] = None
    df = spark.createDataFrame(pdf)
    b = local_batch(df, ["x", "y", "k", "b", "big"])
    x_, y_, k_, b_ = F.col("x"), F.col("y"), F.col("k"), F.col("b")
    exprs = [(x_ * 2.0 + y_) / (k_ - 1.0), (x_ + 0.5) % (k_ * 1.0),
             F.exp(F.log(F.abs(x_) + 1.0)) - F.log1p(y_ * 1.0) + F.sqrt(x_ * 1.0) * F.log10(k_ * 1.0),
             ((x_ > 0) & (y_ < 0.5)) | ~(k_ == 2),
             F.when(x_ > 1.0, x_ * 2.0).when(k_ < 0, y_ * 1.0).otherwise(-1.0) + 0.0,
             F.when(b_, k_ * 1.0).when(x_ < 0, 3.0) * 2.0,
             (x_ * 3.0).cast("int") + (y_ * 1.0).cast("float") * 0.5,
             ((x_ * 10.0).cast("long") + 1.0).cast("double") * k_.cast("double"),
             F.round(x_ * 1.0, 2) + F.floor(y_ * 3.0) - F.ceil(x_ * 1.0) + F.signum(x_ * 1.0),
             F.isnull(x_ * 1.0) | F.isnan(x_ * 2.0) | (F.col("big") * 1.0 > 5e5),
             F.pow(F.abs(x_) * 1.0, 0.5) + F.sin(x_ * 1.0) * F.cos(y_ * 1.0)]
    for e in exprs:
        prog = fused._program(e._expr, b)
        assert prog is not None, str(e._expr)
        got = fused.interpret(prog[0], prog[1], b)
        ref = e._expr.eval(b, EvalContext(spark))
        gm, rm = got.valid_mask().numpy(), ref.valid_mask().numpy()
        assert np.array_equal(gm, rm), str(e._expr)
        gv, rv = got.values.double().numpy()[gm], ref.values.double().numpy()[rm]
        # libm transcendentals may differ in the last ulp; everything else is exact
        assert np.allclose(gv, rv, rtol=1e-12, atol=1e-300, equal_nan=True), str(e._expr)


def test_fused_long_inputs_above_2p53(spark):
    """64-bit integers above 2^53 (monotonically_increasing_id on rank >= 1) must not pass through the
    fp64 operand stack where the result keeps them as longs; where they do fuse (double arithmetic, the same
    long -> double promotion Spark applies) the host reference of the kernel equals the operator path."""
    from cdnaml.models.util import local_batch
    from cdnaml.sql import fused
    from cdnaml.sql import functions as F
    from cdnaml.sql.column import EvalContext
    base = (1 << 33) * 3 + (1 << 53)
    ids = base + np.arange(5000, dtype=np.int64)            # odd ids are not representable in fp64
    pdf = pd.DataFrame({"id": ids, "x": np.linspace(-2, 2, 5000), "k": np.arange(5000).astype(np.int32)})
    df = spark.createDataFrame(pdf)
    b = local_batch(df, ["id", "x", "k"])
    i_, x_, k_ = F.col("id"), F.col("x"), F.col("k")
    refused = [F.when(x_ > 0, i_).otherwise(-1),            # a CASE value keeps the long
               F.when(x_ > 0, i_ * 1.0).otherwise(i_),
               (i_ * 1.0 > 0) & (i_ == i_ + 0),            # long == long
               ((x_ > 0) & (i_ == int(base + 1))),          # long == a literal above 2^53
               (i_ % 7 + x_).cast("int"),                   # hmm: long % int is long arithmetic
               (i_ * 1.0).cast("long") + 0,
               i_.cast("int") + x_,                         # long -> int cast through fp64
               F.abs(i_) + x_]
    for e in refused:
        assert fused._program(e._expr, b) is None, str(e._expr)
    ok = [i_ / 1000.0 + x_, (i_ * 1.0 > 1e3) & (x_ > 0), F.log(i_ * 1.0) + x_, i_.cast("double") * 2.0 - x_,
          (k_ < 100) | (i_ * 1.0 > x_)]
    for e in ok:
        prog = fused._program(e._expr, b)
        assert prog is not None, str(e._expr)
        got = fused.interpret(prog[0], prog[1], b)
        ref = e._expr.eval(b, EvalContext(spark))
        assert np.array_equal(got.values.double().numpy(), ref.values.double().numpy()), str(e._expr)
    # end to end: the operator path keeps odd ids exact
    out = df.select(F.when(x_ > 0, i_).otherwise(-1).alias("v")).toPandas().v.to_numpy()
    np.testing.assert_array_equal(out, np.where(pdf.x > 0, ids, -1))


@pytest.fixture
def spark(tmp_path):
    """Host-reference tests of the expression compiler: a CPU session only (the kernel itself runs in
    tests/test_kernels_gpu.py)."""
    import cdnaml
    from tests.conftest import session_device
    with session_device("cpu"):
        s = cdnaml.SparkSession.builder.config("cdnaml.warehouse.dir", str(tmp_path / "warehouse")).getOrCreate()
        yield s
        s.stop()
