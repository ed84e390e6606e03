"""Instrument the oracle's LLVM IR with FP64 operation counters (test infrastructure).

Reads the textual IR of oracle/grmonty_oracle.cpp (clang -O1, no vectorisation, no FP
contraction) and inserts, after every double-precision arithmetic instruction and every libm
call on doubles, an increment of one slot of the external counter array __grmo_fpc[32]
(defined in fpcount.c).  The counted build then runs the oracle's own track_super_photon
restatement unchanged, so the counts are the exact dynamic FP64 operation counts of the
restatement (tools/count_fp64.py divides them by the transport steps).

    python instrument_ir.py in.ll out.ll
"""
import re
import sys

# counter slots (keep in sync with fpcount.c / tools/count_fp64.py)
SLOTS = {"fadd": 0, "fsub": 1, "fmul": 2, "fdiv": 3, "sqrt": 4, "fma": 5, "fcmp": 6, "cvt": 7,
         "exp": 8, "log": 9, "log10": 10, "pow": 11, "sin": 12, "cos": 13, "acos": 14, "cbrt": 15,
         "tgamma": 16, "other_libm": 17, "exp10": 18, "sincos": 19}
LIBM = {"exp": "exp", "log": "log", "log10": "log10", "pow": "pow", "sin": "sin", "cos": "cos", "acos": "acos",
        "cbrt": "cbrt", "tgamma": "tgamma", "sqrt": "sqrt", "exp10": "exp10", "sincos": "sincos",
        "llvm.exp.f64": "exp", "llvm.log.f64": "log", "llvm.log10.f64": "log10", "llvm.pow.f64": "pow",
        "llvm.sin.f64": "sin", "llvm.cos.f64": "cos", "llvm.sqrt.f64": "sqrt", "llvm.fma.f64": "fma",
        "llvm.fmuladd.f64": "fma", "llvm.exp10.f64": "exp10", "llvm.sincos.f64": "sincos",
        "llvm.acos.f64": "acos"}
ARITH = re.compile(r"^\s*%[\w.]+ = (fadd|fsub|fmul|fdiv)( [a-z ]+)? double ")
FCMP = re.compile(r"^\s*%[\w.]+ = fcmp( [a-z]+)? \w+ double ")
CVT = re.compile(r"^\s*%[\w.]+ = (sitofp|uitofp|fptosi|fptoui) \w+ %?[\w.]+ to (double|i\d+)")
CALL = re.compile(r"^\s*(?:%[\w.]+ = )?(?:tail |musttail |notail )?call [^@]*@([\w.]+)\(")


def slot_of(line):
    m = ARITH.match(line)
    if m:
        return SLOTS[m.group(1)]
    if FCMP.match(line):
        return SLOTS["fcmp"]
    m = CVT.match(line)
    if m and (" double" in line):
        return SLOTS["cvt"]
    m = CALL.match(line)
    if m and m.group(1) in LIBM and "double" in line.split("@")[0] + line:
        return SLOTS[LIBM[m.group(1)]]
    return None


def main(src, dst):
    out, n = [], 0
    for line in open(src):
        out.append(line)
        s = slot_of(line)
        if s is None:
            continue
        gep = f"getelementptr inbounds ([32 x i64], ptr @__grmo_fpc, i64 0, i64 {s})"
        out.append(f"  %__fpc.l{n} = load i64, ptr {gep}, align 8\n")
        out.append(f"  %__fpc.a{n} = add i64 %__fpc.l{n}, 1\n")
        out.append(f"  store i64 %__fpc.a{n}, ptr {gep}, align 8\n")
        n += 1
    out.append("@__grmo_fpc = external global [32 x i64]\n")
    open(dst, "w").writelines(out)
    print(f"instrumented {n} FP64 sites", file=sys.stderr)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
