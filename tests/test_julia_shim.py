"""julia/GPARatScaleHIP.jl against include/gpar_hip.h (CPU only: Julia is absent from this image).

The shim cannot run here, so its binding is checked statically:
* struct GparProblem / GparFitOptions: field names, order and widths equal the header's structs;
* every `ccall((:sym, libgpar), R, (T...), args...)`: the symbol is declared in the header, the
  return and argument types are the Julia equivalents of the C prototype, and the call passes as
  many arguments as the tuple declares;
* the five replaced functions keep the reference's positional arguments and keywords
  (src/gp/dtc.jl:11-25,83-91, gpar_scaled_inference.jl:20-36,141-152,
  temporal_gp_inference.jl:45-54), and the helpers it imports are ones src/util.jl:5-11 exports.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "julia", "GPARatScaleHIP.jl")
HEADER = os.path.join(ROOT, "include", "gpar_hip.h")


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", "", s, flags=re.S)


def _header():
    return _strip_c_comments(open(HEADER).read())


def _c_struct(name):
    m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), _header(), re.S)
    fields = []
    for decl in m.group(1).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        typ, field = decl.rsplit(None, 1)
        if field.startswith("*"):
            typ, field = typ + "*", field[1:]
        fields.append((field, " ".join(typ.split())))
    return fields


def _c_prototypes():
    protos = {}
    for m in re.finditer(r"(\w[\w\s\*]*?)\s*\b(gpar_\w+)\s*\(([^;{]*?)\)\s*;", _header(), re.S):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3)
        params = []
        if args.strip() != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                pm = re.match(r"(.*?)\s*(\w+)$", a)
                params.append(pm.group(1).replace(" *", "*").strip())
        protos[name] = (" ".join(ret.split()), params)
    return protos


C_TO_JL = {
    "int64_t": {"Int64"}, "int32_t": {"Int32"}, "uint64_t": {"UInt64"},
    "const double*": {"Ptr{Float64}"}, "double*": {"Ptr{Float64}"},
    "int32_t*": {"Ptr{Int32}"}, "int64_t*": {"Ptr{Int64}"},
    "const int32_t*": {"Ptr{Int32}", "Ref{Int32}"}, "const int64_t*": {"Ptr{Int64}", "Ref{Int64}"},
    "gpar_ctx*": {"Ptr{Cvoid}"}, "const gpar_ctx*": {"Ptr{Cvoid}"},
    "gpar_ctx**": {"Ptr{Ptr{Cvoid}}"},
    "const gpar_problem*": {"Ref{GparProblem}", "Ptr{GparProblem}"},
    "const gpar_fit_options*": {"Ref{GparFitOptions}", "Ptr{GparFitOptions}"},
    "const double* const*": {"Ref{Ptr{Float64}}", "Ptr{Ptr{Float64}}"},
    "double* const*": {"Ref{Ptr{Float64}}", "Ptr{Ptr{Float64}}"},
    "const char*": {"Cstring", "Ptr{UInt8}"},
    "void*": {"Ptr{Cvoid}"},
}
FIELD_C_TO_JL = {"int64_t": "Int64", "int32_t": "Int32", "double": "Float64",
                 "const double*": "Ptr{Float64}"}


def _split_top(s):
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        out.append("".join(cur).strip())
    return out


def _balanced(s, i):
    """s[i] == '(' -> contents up to the matching ')'."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return s[i + 1:j]
    raise ValueError("unbalanced")


def _shim():
    src = open(SHIM).read()
    return re.sub(r"#=.*?=#", "", src, flags=re.S)


def _ccalls():
    src = _shim()
    calls = []
    for m in re.finditer(r"ccall\(", src):
        parts = _split_top(_balanced(src, m.end() - 1))
        sym = re.match(r"\(:(\w+),\s*libgpar\)", parts[0]).group(1)
        ret = parts[1]
        tup = parts[2].strip()
        assert tup.startswith("(") and tup.endswith(")")
        types = [t for t in _split_top(tup[1:-1]) if t]
        calls.append((sym, ret, types, parts[3:]))
    return calls


def _jl_struct(name):
    m = re.search(r"struct %s\n(.*?)\nend" % name, _shim(), re.S)
    return [tuple(x.strip().split("::")) for x in m.group(1).strip().splitlines()]


@pytest.mark.parametrize("jl,c", [("GparProblem", "gpar_problem"),
                                  ("GparFitOptions", "gpar_fit_options")])
def test_struct_layout_matches_header(jl, c):
    cf = _c_struct(c)
    jf = _jl_struct(jl)
    assert [f for f, _ in jf] == [f for f, _ in cf]
    assert [t for _, t in jf] == [FIELD_C_TO_JL[t] for _, t in cf]


def test_every_ccall_matches_its_prototype():
    protos = _c_prototypes()
    calls = _ccalls()
    assert len(calls) >= 10
    for sym, ret, types, args in calls:
        assert sym in protos, f"{sym} is not declared in include/gpar_hip.h"
        cret, cparams = protos[sym]
        assert ret in C_TO_JL.get(cret, {"?"}) | ({"Int32"} if cret == "int32_t" else set()), (sym, ret, cret)
        assert len(types) == len(cparams), (sym, types, cparams)
        for jt, ct in zip(types, cparams):
            assert jt in C_TO_JL[ct], (sym, jt, ct)
        assert len(args) == len(types), (sym, len(args), len(types))


def test_shim_binds_the_hot_path_entry_points():
    syms = {c[0] for c in _ccalls()}
    for s in ("gpar_dtc_objective", "gpar_dtc_objective_A", "gpar_fit", "gpar_q_u",
              "gpar_fit_predict", "gpar_predict", "gpar_sde_predictions", "gpar_ctx_create",
              "gpar_last_error", "gpar_abi_version"):
        assert s in syms, s


# The reference's signatures (names only): positional arguments and keywords.
REFERENCE_SIGNATURES = {
    # src/gp/dtc.jl:11-25
    "get_optim_scaled_gpar_params": (
        ["input_locations", "pseudo_input_locations", "time_loc", "outputs"],
        ["out_kernel", "time_kernel", "i_log_time_l", "i_log_time_var", "i_log_out_l",
         "i_log_out_var", "i_log_noise_sigma", "optimization_time_limit",
         "show_optimization_trace", "debug", "storage"]),
    # src/gp/dtc.jl:83-91
    "compute_gpar_dtc_objective": (["f", "u", "time_loc", "outputs"],
                                   ["time_kernel", "temporal_noise_sigma", "storage"]),
    # src/gp/gpar_scaled_inference.jl:141-152
    "compute_q_u": (["input_locations", "pseudo_input_locations", "time_loc", "outputs"],
                    ["out_kernel", "time_kernel", "temporal_noise_sigma", "debug", "storage"]),
    # src/gp/gpar_scaled_inference.jl:20-36
    "get_gpar_scaled_predictions": (
        ["input_locations", "pseudo_input_locations", "time_loc", "outputs",
         "inference_time_loc", "inference_input_locations"],
        ["out_kernel_structure", "time_kernel_structure", "i_log_time_l", "i_log_time_var",
         "i_log_out_l", "i_log_out_var", "i_log_noise_sigma", "optimization_time_limit", "debug",
         "storage"]),
    # src/gp/temporal_gp_inference.jl:45-54
    "get_sde_predictions": (["data_locations", "data_outputs", "output_locations"],
                            ["kernel_structure", "sde_storage", "i_log_time_l", "i_log_time_var",
                             "i_log_noise_sigma", "debug"]),
}
# src/util.jl:5-11 exports; temporal_gp_inference.jl:8 exports create_lgssm
REFERENCE_HELPERS = {"to_ColVecs", "unpack_gp", "unpack_gpar", "get_time_mask", "get_output_mask",
                     "parse_initial_gp_params", "parse_initial_gpar_params", "create_lgssm"}


def _jl_function(name):
    src = _shim()
    m = re.search(r"^function %s\(" % name, src, re.M)
    assert m, name
    body = _balanced(src, m.end() - 1)
    pos, _, kw = body.partition(";")
    names = lambda s: [re.match(r"\s*(\w+)", a).group(1) for a in _split_top(s) if a.strip()]
    return names(pos), names(kw)


@pytest.mark.parametrize("name", sorted(REFERENCE_SIGNATURES))
def test_signatures_keep_the_reference_arguments(name):
    pos, kw = _jl_function(name)
    rpos, rkw = REFERENCE_SIGNATURES[name]
    assert pos == rpos
    assert set(rkw) <= set(kw), set(rkw) - set(kw)


def test_helpers_are_the_reference_exports():
    src = _shim()
    used = set(re.findall(r"using GPARatScale: ([\w,\s]+?)\n\n", src, re.S)[0].replace("\n", " ")
               .replace(" ", "").split(","))
    assert used <= REFERENCE_HELPERS, used - REFERENCE_HELPERS
    assert "parse_initial_params" not in src          # not a reference function
    for mod in ("using LinearAlgebra", "using Distributions: MvNormal"):
        assert mod in src


def test_returns_follow_the_reference():
    src = _shim()
    assert "return out[1], A" in src                               # dtc.jl:127 (dtc, A)
    assert "return MvNormal(me, Symmetric(cov)), UpperTriangular(U)" in src   # :185,196
    assert "return opt_lgssm, [Marginal(" in src                   # temporal_gp_inference.jl:113
    assert "return means, stds" in src                             # gpar_scaled_inference.jl:135


def test_multi_output_driver_binds_the_batched_entry_points():
    """get_gpar_scaled_predictions_batch: the reference's per-output driver loop
    (GPAR_scaled_examples.jl:132-175, eeg.jl:212-281) as one gpar_fit_predict_chain (chained
    inference inputs) or gpar_fit_predict call, taking the reference call's positional arguments
    per output and its fit keywords."""
    src = _shim()
    m = re.search(r"^function get_gpar_scaled_predictions_batch\(", src, re.M)
    assert m
    body = src[m.start():src.index("\nend\n", m.start())]
    syms = [c[0] for c in _ccalls() if c[0] in body and f"(:{c[0]}, libgpar)" in body]
    assert "gpar_fit_predict_chain" in syms and "gpar_fit_predict" in syms
    pos, kw = _jl_function("get_gpar_scaled_predictions_batch")
    assert pos == REFERENCE_SIGNATURES["get_gpar_scaled_predictions"][0]
    for k in ("i_log_time_l", "i_log_time_var", "i_log_out_l", "i_log_out_var", "i_log_noise_sigma",
              "optimization_time_limit", "debug", "chained"):
        assert k in kw, k
    assert "get_gpar_scaled_predictions_batch" in re.search(r"export ([\w,\s]+)\n", src).group(1)
    assert "return means, stds" in body


def test_prediction_modes_map_explicitly():
    """every gpar_predict_mode the header declares has a Julia constant of the same
    value, and the mode keyword maps :analytic / :mc / :path explicitly (anything else is a
    DomainError, not a silent ANALYTIC)."""
    src = open(SHIM).read()
    enum = re.search(r"typedef enum gpar_predict_mode \{(.*?)\}", _header(), re.S).group(1)
    c_vals = dict(re.findall(r"(GPAR_PREDICT_\w+)\s*=\s*(\d+)", enum))
    names = re.search(r"const (GPAR_PREDICT_\w+(?:, GPAR_PREDICT_\w+)*) = (.*)", src)
    jl_vals = dict(zip([n.strip() for n in names.group(1).split(",")],
                       re.findall(r"Int32\((\d+)\)", names.group(2))))
    assert jl_vals == c_vals
    body = re.search(r"function predict_mode\(mode::Symbol\)(.*?)\nend", src, re.S).group(1)
    for sym, const in ((":mc", "GPAR_PREDICT_MC"), (":analytic", "GPAR_PREDICT_ANALYTIC"),
                       (":path", "GPAR_PREDICT_PATH")):
        assert f"mode === {sym} && return {const}" in body
    assert "throw(DomainError(mode" in body
    assert "mode === :mc ? " not in src
    assert src.count("md = predict_mode(mode)") == 3


def test_matrix_batch_driver_passes_one_shared_input_matrix():
    """the Julia batch driver's matrix form passes ONE point-major copy of the
    N x P outputs (every output's inputs a column prefix, ldv = P) and one of the N* x P inference
    inputs, which the library's host mode uploads once (prepare_batch / the staged test inputs)."""
    src = open(SHIM).read()
    m = re.search(r"function get_gpar_scaled_predictions_batch\(Y::AbstractMatrix,(.*?)\nend\n", src, re.S)
    assert m, "matrix form missing"
    body = m.group(1)
    assert "Yt = Matrix{Float64}(permutedims(Y))" in body
    assert "GparProblem(N, size(Zs[i - 1], 2), i - 1, pointer(t), pointer(Yt), P," in body
    assert "vptr = fill(pointer(Ft), Q)" in body and "lds = fill(Int64(P), Q)" in body
    assert body.count("ccall((:gpar_fit_predict") == 2
