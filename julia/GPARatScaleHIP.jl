#=
GPARatScaleHIP -- the reference's scaled-GPAR hot path on MI355X through libgparhip.so.

A drop-in for the functions of GPARatScale's hot path (BASELINE.json north_star): same names,
positional arguments, keywords and return shapes as

  compute_gpar_dtc_objective    src/gp/dtc.jl:83-128          -> (dtc, A)
  get_optim_scaled_gpar_params  src/gp/dtc.jl:11-77           -> (time_l, time_var, out_l, out_var, noise_sigma)
  compute_q_u                   src/gp/gpar_scaled_inference.jl:141-196 -> (q_u::MvNormal, U_u)
  get_gpar_scaled_predictions   src/gp/gpar_scaled_inference.jl:20-136  -> (means, stds)
  get_sde_predictions           src/gp/temporal_gp_inference.jl:45-114  -> (lgssm, marginals)

and adds the multi-output driver the reference writes as a loop in its examples
(GPAR_scaled_examples.jl:132-175, eeg.jl:212-281):

  get_gpar_scaled_predictions_batch  -> (means, stds), one vector per output, one library call

with every number computed by the gfx950 kernels behind include/gpar_hip.h.  A caller switches
`using GPARatScale` to `using GPARatScale, GPARatScaleHIP` and qualifies these five names (or
imports them from GPARatScaleHIP).  The reference's helpers (to_ColVecs, unpack_gpar,
unpack_gp, parse_initial_gpar_params, parse_initial_gp_params, create_lgssm) are used as they are.

Julia is absent from the image this was written in, so this file has not been run; its ccall
argument tuples and struct layouts are checked against include/gpar_hip.h by
tests/test_julia_shim.py.  Stheno kernel introspection (_kernel_params) follows the Stheno
0.6-era types the reference's `kernel(k; l, s)` builds (SURVEY §8c: versions unpinned).
=#
module GPARatScaleHIP

using LinearAlgebra
using Random
using Distributions: MvNormal
using Stheno
using Stheno: Matern12, Matern32, Matern52, EQ
using TemporalGPs: SArrayStorage
import GPARatScale
using GPARatScale: to_ColVecs, unpack_gpar, unpack_gp, parse_initial_gpar_params,
                   parse_initial_gp_params

export compute_gpar_dtc_objective, get_optim_scaled_gpar_params, compute_q_u,
       get_gpar_scaled_predictions, get_sde_predictions, get_gpar_scaled_predictions_batch

const libgpar = get(ENV, "GPAR_HIP_LIB", "libgparhip.so")

# ------------------------------------------------------------------ include/gpar_hip.h constants
const GPAR_ABI_VERSION = Int32(1)
const GPAR_OK, GPAR_ERR_ARG, GPAR_ERR_NOT_PD = Int32(0), Int32(1), Int32(2)
const GPAR_MEM_HOST = Int32(0)
const GPAR_PREDICT_ANALYTIC, GPAR_PREDICT_MC, GPAR_PREDICT_PATH = Int32(0), Int32(1), Int32(2)

# prediction estimator: :mc (the reference's, gpar_scaled_inference.jl:110-130), :analytic (its
# S -> infinity limit) or :path (tmp.jl:119-167, posterior_rand paths); anything else is an error
function predict_mode(mode::Symbol)
    mode === :mc && return GPAR_PREDICT_MC
    mode === :analytic && return GPAR_PREDICT_ANALYTIC
    mode === :path && return GPAR_PREDICT_PATH
    throw(DomainError(mode, "mode must be :mc, :analytic or :path"))
end

kernel_id(::Matern12) = Int32(0)
kernel_id(::Matern32) = Int32(1)
kernel_id(::Matern52) = Int32(2)
kernel_id(::EQ) = Int32(3)

# struct gpar_problem (field order and widths as in the header)
struct GparProblem
    n::Int64
    m::Int64
    d::Int64
    t::Ptr{Float64}
    v::Ptr{Float64}
    ldv::Int64
    z::Ptr{Float64}
    ldz::Int64
    y::Ptr{Float64}
    out_kernel::Int32
    time_kernel::Int32
    kuu_noise::Int32
    mem::Int32
    qu_kuu_noise::Int32
end

# struct gpar_fit_options
struct GparFitOptions
    max_evals::Int32
    max_iterations::Int32
    g_tol::Float64
    time_limit::Float64
end

# ------------------------------------------------------------------ context and errors
mutable struct Ctx
    h::Ptr{Cvoid}
    function Ctx(device::Integer = 0)
        v = ccall((:gpar_abi_version, libgpar), Int32, ())
        v == GPAR_ABI_VERSION || error("libgparhip ABI $v, this binding expects $GPAR_ABI_VERSION")
        r = Ref{Ptr{Cvoid}}(C_NULL)
        st = ccall((:gpar_ctx_create, libgpar), Int32, (Int32, Ptr{Ptr{Cvoid}}), device, r)
        st == GPAR_OK || error("gpar_ctx_create($device) failed ($st): no MI355X visible?")
        c = new(r[])
        finalizer(c) do c
            ccall((:gpar_ctx_destroy, libgpar), Int32, (Ptr{Cvoid},), c.h)
        end
    end
end

const CTX = Ref{Union{Nothing,Ctx}}(nothing)
ctx() = something(CTX[], (CTX[] = Ctx(parse(Int, get(ENV, "GPAR_HIP_DEVICE", "0")))))

function check(c::Ctx, st)
    st == GPAR_OK && return nothing
    msg = unsafe_string(ccall((:gpar_last_error, libgpar), Cstring, (Ptr{Cvoid},), c.h))
    st == GPAR_ERR_NOT_PD && throw(PosDefException(0))      # as `cholesky` at dtc.jl:119-120
    st == GPAR_ERR_ARG && throw(DomainError(msg))            # as util.jl:112-117
    error("libgparhip: $msg")
end

# ------------------------------------------------------------------ Stheno objects -> numbers
# kernel(k; l, s) (Stheno 0.6) builds s * stretch(k, 1 / l): Scaled{σ², Stretched{a, base}}.
_base(k::Union{Matern12,Matern32,Matern52,EQ}) = (k, 1.0, 1.0)
function _base(k::Stheno.Stretched)
    b, a, s = _base(k.k)
    return b, a * only(k.a), s
end
function _base(k::Stheno.Scaled)
    b, a, s = _base(k.k)
    return b, a, s * only(k.σ²)
end
"(structure, lengthscale l, variance s) of kernel(structure; l, s)."
function _kernel_params(k)
    b, a, s = _base(k)
    return b, 1.0 / a, s
end

# ColVecs (util.jl:16-31) is D x N column-major: point k is column k, so ldv = D.
_colmat(x) = Matrix{Float64}(to_ColVecs(x).X)

function problem(V::Matrix{Float64}, Z::Matrix{Float64}, t::Vector{Float64}, y::Vector{Float64},
                 out_kernel, time_kernel; kuu_noise::Bool = true, qu_kuu_noise::Bool = false)
    size(V, 1) == size(Z, 1) || throw(DomainError(size(Z, 1), "V and Z dimensions differ"))
    length(t) == length(y) == size(V, 2) || throw(DomainError(length(t), "t, y, V lengths differ"))
    return GparProblem(length(t), size(Z, 2), size(V, 1), pointer(t), pointer(V), size(V, 1),
                       pointer(Z), size(Z, 1), pointer(y), kernel_id(out_kernel),
                       kernel_id(time_kernel), Int32(kuu_noise), GPAR_MEM_HOST, Int32(qu_kuu_noise))
end

# Optim.Options(time_limit = ...) of dtc.jl:58-61: iterations 1000, g_tol 1e-8, no eval budget
fit_options(time_limit) = GparFitOptions(Int32(0), Int32(1000), 1e-8, Float64(time_limit))

# ------------------------------------------------------------------ dtc.jl:83-128
"""
compute_gpar_dtc_objective(f, u, time_loc, outputs; time_kernel, temporal_noise_sigma, storage)

f = GP(k_o)(V, σ²) and u = GP(k_o)(Z, σ²) as get_optim_scaled_gpar_params builds them
(dtc.jl:35-36).  Returns (dtc, A) like dtc.jl:127; A (M x N) is materialised only with
`materialize_A = true` (every caller in the reference discards it), else `nothing`.
"""
function compute_gpar_dtc_objective(f, u, time_loc, outputs;
                                    time_kernel = Matern52(), temporal_noise_sigma = 0.04,
                                    storage = SArrayStorage(Float64), materialize_A::Bool = false)
    ok, l_o, s_o = _kernel_params(f.f.k)
    tk, l_t, s_t = _kernel_params(time_kernel)
    σ = Float64(temporal_noise_sigma)
    # the library adds σ² to cov(u) itself (dtc.jl:35,119: u = gp_prior(Z, noise_sigma^2))
    all(≈(σ^2), diag(u.Σy)) || throw(ArgumentError("cov(u) jitter must be temporal_noise_sigma^2"))
    V, Z = _colmat(f.x), _colmat(u.x)
    t = Vector{Float64}(time_loc)
    y = Vector{Float64}(outputs .- mean(f))                  # dtc.jl:106 decorrelates outputs - mean(f)
    th = [l_t, sqrt(s_t), l_o, sqrt(s_o), σ]                  # natural units, variances squared inside
    c = ctx()
    out = zeros(1)
    A = materialize_A ? zeros(size(Z, 2), length(t)) : nothing
    GC.@preserve V Z t y th begin
        p = Ref(problem(V, Z, t, y, ok, tk))
        if materialize_A
            check(c, ccall((:gpar_dtc_objective_A, libgpar), Int32,
                           (Ptr{Cvoid}, Ref{GparProblem}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                           c.h, p, th, out, A))
        else
            check(c, ccall((:gpar_dtc_objective, libgpar), Int32,
                           (Ptr{Cvoid}, Ref{GparProblem}, Int32, Ptr{Float64}, Ptr{Float64}),
                           c.h, p, Int32(1), th, out))
        end
    end
    return out[1], A
end

# ------------------------------------------------------------------ dtc.jl:11-77
function get_optim_scaled_gpar_params(input_locations, pseudo_input_locations, time_loc, outputs;
        out_kernel = Matern52(), time_kernel = Matern52(),
        i_log_time_l = nothing, i_log_time_var = nothing, i_log_out_l = nothing,
        i_log_out_var = nothing, i_log_noise_sigma = nothing,
        optimization_time_limit = 1000.0, show_optimization_trace = false, debug::Bool = false,
        storage = SArrayStorage(Float64))
    # show_optimization_trace and storage are accepted for signature parity: the simplex runs
    # inside the library (nelder_mead.hpp) and the state-space storage is the kernels' own.
    V = _colmat(input_locations)
    Z = _colmat(pseudo_input_locations)
    t = Vector{Float64}(time_loc)
    y = Vector{Float64}(outputs)
    x0 = Vector{Float64}(parse_initial_gpar_params(i_log_time_l, i_log_time_var, i_log_out_l,
                                                   i_log_out_var, i_log_noise_sigma))
    if debug
        i_time_l, i_time_var, i_out_l, i_out_var, i_noise_sigma = unpack_gpar(x0)
        println("Generating scaled GPAR with initial parameters:")
        println("\ti_time_l=$(i_time_l); i_time_var=$(i_time_var); i_out_l=$(i_out_l); i_out_var=$(i_out_var); i_noise_sigma=$(i_noise_sigma)")
    end
    c = ctx()
    θ = zeros(5)
    nlml = zeros(1)
    ev = zeros(Int32, 1)
    opts = Ref(fit_options(optimization_time_limit))
    GC.@preserve V Z t y x0 begin
        p = Ref(problem(V, Z, t, y, out_kernel, time_kernel))
        check(c, ccall((:gpar_fit, libgpar), Int32,
                       (Ptr{Cvoid}, Ref{GparProblem}, Int32, Ptr{Float64}, Ref{GparFitOptions},
                        Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                       c.h, p, Int32(1), x0, opts, θ, nlml, ev))
    end
    opt_params = Tuple(θ)
    if debug
        println("Finished optimizing parameters:")
        println("\tOptimum time L: $(θ[1]) ")
        println("\tOptimum time var: $(θ[2])")
        println("\tOptimum outputs l: $(θ[3])")
        println("\tOptimum outputs var: $(θ[4])")
        println("\tOptimum Noise std: $(θ[5])")
        println()
    end
    return opt_params
end

# ------------------------------------------------------------------ gpar_scaled_inference.jl:141-196
function compute_q_u(input_locations, pseudo_input_locations, time_loc, outputs;
                     out_kernel = Matern52(), time_kernel = Matern52(),
                     temporal_noise_sigma = 0.05, debug::Bool = false,
                     storage = SArrayStorage(Float64))
    ok, l_o, s_o = _kernel_params(out_kernel)
    tk, l_t, s_t = _kernel_params(time_kernel)
    V = _colmat(input_locations)
    Z = _colmat(pseudo_input_locations)
    t = Vector{Float64}(time_loc)
    y = Vector{Float64}(outputs)
    th = [l_t, sqrt(s_t), l_o, sqrt(s_o), Float64(temporal_noise_sigma)]
    M = size(Z, 2)
    me = zeros(M)
    cov = zeros(M, M)
    U = zeros(M, M)
    c = ctx()
    GC.@preserve V Z t y th begin
        p = Ref(problem(V, Z, t, y, ok, tk))
        check(c, ccall((:gpar_q_u, libgpar), Int32,
                       (Ptr{Cvoid}, Ref{GparProblem}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                        Ptr{Float64}),
                       c.h, p, th, me, cov, U))
    end
    return MvNormal(me, Symmetric(cov)), UpperTriangular(U)
end

# ------------------------------------------------------------------ gpar_scaled_inference.jl:20-136
"""
Same signature and result as the reference: the fit (Matern52 for both kernels, as :48-49
hard-codes), q(u) and the 100-sample Monte Carlo at the inference locations.  Extra keywords:
`mode = :mc` (the reference's estimator) or `:analytic` (its S -> infinity limit), `samples`,
`seed` (default: drawn from the global RNG, so repeated calls vary as the reference's do).
"""
function get_gpar_scaled_predictions(input_locations, pseudo_input_locations, time_loc, outputs,
        inference_time_loc, inference_input_locations;
        out_kernel_structure = Matern52(), time_kernel_structure = Matern52(),
        i_log_time_l = nothing, i_log_time_var = nothing, i_log_out_l = nothing,
        i_log_out_var = nothing, i_log_noise_sigma = nothing,
        optimization_time_limit = 1000.0, debug::Bool = false,
        storage = SArrayStorage(Float64),
        mode::Symbol = :mc, samples::Integer = 100, seed::UInt64 = rand(UInt64))
    V = _colmat(input_locations)
    Z = _colmat(pseudo_input_locations)
    Vs = _colmat(inference_input_locations)
    t = Vector{Float64}(time_loc)
    y = Vector{Float64}(outputs)
    ts = Vector{Float64}(inference_time_loc)
    md = predict_mode(mode)
    x0 = Vector{Float64}(parse_initial_gpar_params(i_log_time_l, i_log_time_var, i_log_out_l,
                                                   i_log_out_var, i_log_noise_sigma))
    debug && println("Starting optimization")
    c = ctx()
    θ = zeros(5)
    nlml = zeros(1)
    ev = zeros(Int32, 1)
    ns = length(ts)
    means = zeros(ns)
    stds = zeros(ns)
    opts = Ref(fit_options(optimization_time_limit))
    GC.@preserve V Z Vs t y ts x0 θ means stds begin
        pfit = Ref(problem(V, Z, t, y, Matern52(), Matern52()))
        if out_kernel_structure isa Matern52 && time_kernel_structure isa Matern52
            # one call: batched fit, then q(u) and prediction at the fitted theta
            vsp = Ref(pointer(Vs))
            lds = Ref(Int64(size(Vs, 1)))
            mp = Ref(pointer(means))
            sp = Ref(pointer(stds))
            check(c, ccall((:gpar_fit_predict, libgpar), Int32,
                           (Ptr{Cvoid}, Ref{GparProblem}, Int32, Ptr{Float64}, Ref{GparFitOptions},
                            Int64, Ptr{Float64}, Ref{Ptr{Float64}}, Ref{Int64}, Int32, Int32, UInt64,
                            Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ref{Ptr{Float64}},
                            Ref{Ptr{Float64}}),
                           c.h, pfit, Int32(1), x0, opts, ns, ts, vsp, lds, md, Int32(samples),
                           seed, θ, nlml, ev, mp, sp))
        else
            check(c, ccall((:gpar_fit, libgpar), Int32,
                           (Ptr{Cvoid}, Ref{GparProblem}, Int32, Ptr{Float64}, Ref{GparFitOptions},
                            Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                           c.h, pfit, Int32(1), x0, opts, θ, nlml, ev))
            ppred = Ref(problem(V, Z, t, y, out_kernel_structure, time_kernel_structure))
            check(c, ccall((:gpar_predict, libgpar), Int32,
                           (Ptr{Cvoid}, Ref{GparProblem}, Ptr{Float64}, Int64, Ptr{Float64},
                            Ptr{Float64}, Int64, Int32, Int32, UInt64, Ptr{Float64}, Ptr{Float64}),
                           c.h, ppred, θ, ns, ts, Vs, Int64(size(Vs, 1)), md, Int32(samples), seed,
                           means, stds))
        end
    end
    return means, stds
end

# ------------------------------------------------------------------ the GPAR per-output driver loop
"""
    get_gpar_scaled_predictions_batch(input_locations, pseudo_input_locations, time_loc, outputs,
                                      inference_time_loc, inference_input_locations;
                                      chained = true, kwargs...)

The per-output driver loop of examples/GPAR_scaled_examples.jl:132-175 and examples/eeg.jl:212-281
-- one `get_gpar_scaled_predictions` per output -- as ONE library call (gpar_fit_predict_chain /
gpar_fit_predict): the P fits run as one batched Nelder-Mead on the GPU (pipelined, CU-split,
distance-cached), then the predictions in output order.  Output i = 1..P has training inputs
`input_locations[i]`, pseudo-inputs `pseudo_input_locations[i]` and targets `outputs[i]` on the shared
`time_loc`, each as get_gpar_scaled_predictions takes them.

Inference inputs:
* `chained = true` (the reference's loops: y3 reads y2's predicted means,
  GPAR_scaled_examples.jl:172; eeg.jl:249,274): `inference_input_locations` is the list of GIVEN
  inference columns (e.g. `[test_y1]`, or eeg.jl's `[train_f3, train_f4, train_f5, train_f6]`), and
  output i reads the first D_i columns of [given columns..., predicted means of outputs 1..i-1];
* `chained = false`: `inference_input_locations[i]` are output i's own inference inputs.

Initial log-parameters (`i_log_*`) are scalars shared by every output or `nothing` (a fresh
U(0,1) draw per output, as each reference call makes).  Returns (means, stds): P vectors each,
what get_gpar_scaled_predictions returns for that output.
"""
function get_gpar_scaled_predictions_batch(input_locations, pseudo_input_locations, time_loc,
        outputs, inference_time_loc, inference_input_locations;
        chained::Bool = true,
        i_log_time_l = nothing, i_log_time_var = nothing, i_log_out_l = nothing,
        i_log_out_var = nothing, i_log_noise_sigma = nothing,
        optimization_time_limit = 1000.0, debug::Bool = false,
        mode::Symbol = :mc, samples::Integer = 100, seed::UInt64 = rand(UInt64))
    P = length(outputs)
    length(input_locations) == length(pseudo_input_locations) == P ||
        throw(DomainError(P, "one input / pseudo-input set per output"))
    t = Vector{Float64}(time_loc)
    ts = Vector{Float64}(inference_time_loc)
    ns = length(ts)
    Vs = [_colmat(x) for x in input_locations]
    Zs = [_colmat(z) for z in pseudo_input_locations]
    ys = [Vector{Float64}(y) for y in outputs]
    # Matern52 for both kernels, as get_gpar_scaled_predictions hard-codes for its fit (:48-49)
    probs = [problem(Vs[i], Zs[i], t, ys[i], Matern52(), Matern52()) for i in 1:P]
    x0 = reduce(vcat, [Vector{Float64}(parse_initial_gpar_params(i_log_time_l, i_log_time_var,
                       i_log_out_l, i_log_out_var, i_log_noise_sigma)) for _ in 1:P])
    md = predict_mode(mode)
    θ = zeros(5 * P)
    nlml = zeros(P)
    ev = zeros(Int32, P)
    means = [zeros(ns) for _ in 1:P]
    stds = [zeros(ns) for _ in 1:P]
    mptr = [pointer(m) for m in means]
    sptr = [pointer(s) for s in stds]
    opts = Ref(fit_options(optimization_time_limit))
    debug && println("Starting the batched optimization of $P outputs")
    c = ctx()
    if chained
        given = [Vector{Float64}(x) for x in inference_input_locations]
        K = length(given) + P
        all(length(g) == ns for g in given) || throw(DomainError(ns, "inference columns of length N*"))
        # point-major chain: point k's K columns contiguous (chain[k*K + col])
        chain = zeros(K, ns)
        for (j, g) in enumerate(given)
            chain[j, :] .= g
        end
        for i in 1:P
            size(Vs[i], 1) <= length(given) + i - 1 ||
                throw(DomainError(i, "output $i reads $(size(Vs[i], 1)) inference columns, only " *
                                     "$(length(given)) given + $(i - 1) predicted exist before it"))
        end
        cols = Int32[length(given) + i - 1 for i in 1:P]
        vptr = fill(pointer(chain), P)
        lds = fill(Int64(K), P)
        GC.@preserve Vs Zs ys t ts x0 θ nlml ev means stds chain cols probs begin
            check(c, ccall((:gpar_fit_predict_chain, libgpar), Int32,
                           (Ptr{Cvoid}, Ptr{GparProblem}, Int32, Ptr{Float64}, Ref{GparFitOptions},
                            Int64, Ptr{Float64}, Ptr{Ptr{Float64}}, Ptr{Int64}, Int32, Int32, UInt64,
                            Ptr{Float64}, Int64, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32},
                            Ptr{Ptr{Float64}}, Ptr{Ptr{Float64}}),
                           c.h, probs, Int32(P), x0, opts, ns, ts, vptr, lds, md, Int32(samples),
                           seed, chain, Int64(K), cols, θ, nlml, ev, mptr, sptr))
        end
    else
        Vstar = [_colmat(x) for x in inference_input_locations]
        length(Vstar) == P || throw(DomainError(P, "one inference input set per output"))
        vptr = [pointer(v) for v in Vstar]
        lds = Int64[size(v, 1) for v in Vstar]
        GC.@preserve Vs Zs ys t ts x0 θ nlml ev means stds Vstar probs begin
            check(c, ccall((:gpar_fit_predict, libgpar), Int32,
                           (Ptr{Cvoid}, Ptr{GparProblem}, Int32, Ptr{Float64}, Ref{GparFitOptions},
                            Int64, Ptr{Float64}, Ptr{Ptr{Float64}}, Ptr{Int64}, Int32, Int32, UInt64,
                            Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Ptr{Float64}},
                            Ptr{Ptr{Float64}}),
                           c.h, probs, Int32(P), x0, opts, ns, ts, vptr, lds, md, Int32(samples),
                           seed, θ, nlml, ev, mptr, sptr))
        end
    end
    if debug
        for i in 1:P
            println("Output $i: optimum params $(Tuple(θ[5i-4:5i]))")
        end
    end
    return means, stds
end

"""
    get_gpar_scaled_predictions_batch(Y::AbstractMatrix, pseudo_input_locations, time_loc,
                                      inference_time_loc, F::AbstractMatrix; chained = false, kw...)

GPAR's own structure as one matrix (GPAR_scaled_examples.jl:132-175): column i of Y (N x P) is
output i's observed targets, and output i's training inputs are columns 1..i-1 -- so every output's
inputs are column prefixes of ONE matrix, passed once (the library uploads it once) instead of P
copies.  Predicts outputs 2..P (output 1 is the temporal-only get_sde_predictions); output i's
pseudo-inputs are `pseudo_input_locations[i - 1]` (D = i - 1).  Inference inputs: F (N* x P), output
i reads its first i - 1 columns -- as given (`chained = false`), or with `chained = true` F's
column 1 (test_y1) followed by the predicted means of outputs 2..i-1 (GPAR_scaled_examples.jl:172).
Returns (means, stds) for outputs 2..P.
"""
function get_gpar_scaled_predictions_batch(Y::AbstractMatrix, pseudo_input_locations,
        time_loc, inference_time_loc, F::AbstractMatrix;
        chained::Bool = false,
        i_log_time_l = nothing, i_log_time_var = nothing, i_log_out_l = nothing,
        i_log_out_var = nothing, i_log_noise_sigma = nothing,
        optimization_time_limit = 1000.0, debug::Bool = false,
        mode::Symbol = :mc, samples::Integer = 100, seed::UInt64 = rand(UInt64))
    N, P = size(Y)
    P >= 2 || throw(DomainError(P, "Y needs at least two output columns"))
    length(pseudo_input_locations) == P - 1 ||
        throw(DomainError(P, "one pseudo-input set per output 2..P"))
    size(F, 2) == P || throw(DomainError(size(F, 2), "F must have the P columns of Y"))
    t = Vector{Float64}(time_loc)
    ts = Vector{Float64}(inference_time_loc)
    ns = length(ts)
    length(t) == N && size(F, 1) == ns || throw(DomainError(N, "Y / F rows must match the times"))
    # point-major: point k's outputs contiguous, so output i's inputs are a column prefix (ldv = P)
    Yt = Matrix{Float64}(permutedims(Y))
    Ft = Matrix{Float64}(permutedims(F))
    Zs = [_colmat(z) for z in pseudo_input_locations]
    ys = [Vector{Float64}(Y[:, i]) for i in 2:P]
    probs = GparProblem[]
    for i in 2:P
        size(Zs[i - 1], 1) == i - 1 || throw(DomainError(i, "output $i's pseudo-inputs must have $(i - 1) rows"))
        push!(probs, GparProblem(N, size(Zs[i - 1], 2), i - 1, pointer(t), pointer(Yt), P,
                                 pointer(Zs[i - 1]), i - 1, pointer(ys[i - 1]),
                                 kernel_id(Matern52()), kernel_id(Matern52()), Int32(1),
                                 GPAR_MEM_HOST, Int32(0)))
    end
    Q = P - 1
    x0 = reduce(vcat, [Vector{Float64}(parse_initial_gpar_params(i_log_time_l, i_log_time_var,
                       i_log_out_l, i_log_out_var, i_log_noise_sigma)) for _ in 1:Q])
    md = predict_mode(mode)
    θ = zeros(5 * Q)
    nlml = zeros(Q)
    ev = zeros(Int32, Q)
    means = [zeros(ns) for _ in 1:Q]
    stds = [zeros(ns) for _ in 1:Q]
    mptr = [pointer(m) for m in means]
    sptr = [pointer(s) for s in stds]
    vptr = fill(pointer(Ft), Q)
    lds = fill(Int64(P), Q)
    opts = Ref(fit_options(optimization_time_limit))
    c = ctx()
    GC.@preserve Yt Ft Zs ys t ts x0 θ nlml ev means stds probs begin
        if chained
            cols = Int32[i - 1 for i in 2:P]   # output i's mean -> column i (0-based i - 1)
            check(c, ccall((:gpar_fit_predict_chain, libgpar), Int32,
                           (Ptr{Cvoid}, Ptr{GparProblem}, Int32, Ptr{Float64}, Ref{GparFitOptions},
                            Int64, Ptr{Float64}, Ptr{Ptr{Float64}}, Ptr{Int64}, Int32, Int32, UInt64,
                            Ptr{Float64}, Int64, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32},
                            Ptr{Ptr{Float64}}, Ptr{Ptr{Float64}}),
                           c.h, probs, Int32(Q), x0, opts, ns, ts, vptr, lds, md, Int32(samples),
                           seed, Ft, Int64(P), cols, θ, nlml, ev, mptr, sptr))
        else
            check(c, ccall((:gpar_fit_predict, libgpar), Int32,
                           (Ptr{Cvoid}, Ptr{GparProblem}, Int32, Ptr{Float64}, Ref{GparFitOptions},
                            Int64, Ptr{Float64}, Ptr{Ptr{Float64}}, Ptr{Int64}, Int32, Int32, UInt64,
                            Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Ptr{Float64}},
                            Ptr{Ptr{Float64}}),
                           c.h, probs, Int32(Q), x0, opts, ns, ts, vptr, lds, md, Int32(samples),
                           seed, θ, nlml, ev, mptr, sptr))
        end
    end
    if debug
        for i in 1:Q
            println("Output $(i + 1): optimum params $(Tuple(θ[5i-4:5i]))")
        end
    end
    return means, stds
end

# ------------------------------------------------------------------ temporal_gp_inference.jl:45-114
"Marginal of the latent f at one output location: `.m[1]` mean, `.P[1]` variance."
struct Marginal
    m::Vector{Float64}
    P::Matrix{Float64}
end

function get_sde_predictions(data_locations, data_outputs, output_locations;
        kernel_structure::Kernel = Matern52(), sde_storage::SArrayStorage = SArrayStorage(Float64),
        i_log_time_l = nothing, i_log_time_var = nothing, i_log_noise_sigma = nothing,
        debug::Bool = true)
    t = Vector{Float64}(data_locations)
    y = Vector{Float64}(data_outputs)
    ts = Vector{Float64}(output_locations)
    x0 = Vector{Float64}(parse_initial_gp_params(i_log_time_l, i_log_time_var, i_log_noise_sigma))
    θ = zeros(3)
    m = zeros(length(ts))
    v = zeros(length(ts))
    # Optim.optimize(nlml, params, NelderMead()) with default Options (:82)
    opts = Ref(fit_options(0.0))
    c = ctx()
    GC.@preserve t y ts x0 begin
        check(c, ccall((:gpar_sde_predictions, libgpar), Int32,
                       (Ptr{Cvoid}, Int32, Int64, Ptr{Float64}, Ptr{Float64}, Int64, Int64,
                        Ptr{Float64}, Int32, Ptr{Float64}, Ref{GparFitOptions}, Int32,
                        Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                       c.h, Int32(1), length(t), t, y, Int64(length(t)), length(ts), ts,
                       kernel_id(kernel_structure), x0, opts, GPAR_MEM_HOST, θ, m, v))
    end
    opt_l, opt_process_var, opt_noise_sigma = θ
    if debug
        println("Finished optimizing parameters:")
        println("\tOptimum L: $(opt_l) ")
        println("\tOptimum Process Variance: $(opt_process_var)")
        println("\tOptimum noise: $(opt_noise_sigma)")
        println()
    end
    # the model object the reference returns (:97-105), built by its own create_lgssm (no compute)
    latent = vcat(t, ts)
    perm = sortperm(latent)
    noise_vector = vcat(fill(opt_noise_sigma^2, length(t)), fill(1e10, length(ts)))[perm]
    opt_lgssm = GPARatScale.create_lgssm(latent[perm], opt_l, opt_process_var, opt_noise_sigma,
                                         kernel_structure; noise_vector = noise_vector)
    return opt_lgssm, [Marginal([m[k]], fill(v[k], 1, 1)) for k in eachindex(ts)]
end

end # module
