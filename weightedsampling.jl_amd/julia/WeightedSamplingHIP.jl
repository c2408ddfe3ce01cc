"""
    WeightedSamplingHIP

MI355X backend for WeightedSampling.jl: a `HipColumnStore <: AbstractParticleStore`
(src/stores.jl:1-35) plus `apply!` specialisations for `SMCState{<:HipColumnStore}` that
route the per-particle hot path (Sample / Observe / Weight / Assign / Resample / Move) to
`libwsmc.so` through `ccall` (include/wsmc.h). The reference package is not edited: Julia's
dispatch picks these methods because they are more specific in the store type
(src/types.jl:48).

UNTESTED: the build image has no Julia toolchain. Every `ccall` below mirrors a binding of
the Python ctypes layer (`weightedsampling.jl_amd/wsmc/abi.py`), which the test-suite runs
against the same library on MI355X. See INTEGRATION.md.

Device arguments are recognised structurally. `getcol` on a `HipColumnStore` returns a
`DeviceColumn` proxy. Broadcasting `+ - *` over proxies and `Ref` constants (the shapes
`vectorize` emits, src/rewrites.jl:146-219) builds a lazy affine `DeviceExpr`, which
becomes a `wsmc_operand`. Any other fused broadcast over the operators `wsmc_assign_expr`
knows (arithmetic, `^`, `min`/`max`, `abs`, `sqrt`, `exp`, `log`, `log1p`, `sin`, `cos`,
comparisons, `!`, `&`, `|`, `ifelse`) becomes a `DeviceProgram`: an Assign evaluates it on the
device, a distribution argument through a temporary device column. Only a function outside
that set is materialised on the host (download → compute → temporary column).
"""
module WeightedSamplingHIP

using WeightedSampling
using LinearAlgebra: PosDefException, I
using Distributions: Normal, MvNormal, Uniform, Truncated
const WS = WeightedSampling
import WeightedSampling: nparticles, hascol, getcol, colnames, broadcast_setcol!, resample!, apply!,
    log_evidence

export HipColumnStore, lazy!, materialize!, ssm2d_run!, sync_weights!, expectation, describe_device, sample_device, shard!,
       comm_unique_id

const libwsmc = get(ENV, "WSMC_LIB", joinpath(@__DIR__, "..", "wsmc", "libwsmc.so"))

# ---------------------------------------------------------------------------------------
# C structs (include/wsmc.h) — field order and sizes must match (tests/test_abi.py checks
# the C side against the Python mirror; Julia isbits structs follow the same C layout)
# ---------------------------------------------------------------------------------------
struct WsmcOperand
    c0::Float64
    col::NTuple{2,Int32}
    comp::NTuple{2,Int32}
    coef::NTuple{2,Float64}
end
const_operand(v) = WsmcOperand(Float64(v), (Int32(-1), Int32(-1)), (Int32(0), Int32(0)), (0.0, 0.0))

struct WsmcDist
    family::Int32
    mean_fn::Int32
    dim::Int32
    reserved::Int32
    mu::NTuple{4,WsmcOperand}
    scale::WsmcOperand
    param::NTuple{2,Float64}
end

struct WsmcState
    resampled::Int32
    weights_changed::Int32
    depth::Int32
    n_terms::Int32
    last_ess_perc::Float64
    op_counter::UInt64
    n_resamples::Int64
end

struct WsmcXInst            # wsmc_xinst: one instruction of a postfix program
    op::Int32
    col::Int32
    comp::Int32
    reserved::Int32
    c::Float64
end

const WSMC_ENOTPD = 3
const FAM_NORMAL, FAM_HALFNORMAL, FAM_UNIFORM, FAM_MVNORMAL_ISO, FAM_MVNORMAL =
    Int32(0), Int32(1), Int32(2), Int32(3), Int32(4)
# the scalar families from WSMC_FAM_BERNOULLI on: (kernel name, family, location index, scale index)
# into the kernel's argument tuple (0: none)
const EXT_FAMILIES = ((:Bernoulli, 5, 1, 0), (:BernoulliLogit, 6, 1, 0), (:Exponential, 7, 0, 1),
                      (:LogNormal, 8, 1, 2), (:Laplace, 9, 1, 2), (:Cauchy, 10, 1, 2), (:Logistic, 11, 1, 2),
                      (:Gumbel, 12, 1, 2), (:Rayleigh, 13, 0, 1), (:Geometric, 14, 1, 0))
const MEAN_AFFINE = Int32(0)
const RESAMPLE_STRATIFIED = Int32(0)
const PROPOSAL_RW, PROPOSAL_AUTORW = Int32(0), Int32(1)

function check(rc::Integer)
    rc == 0 && return nothing
    msg = unsafe_string(ccall((:wsmc_last_error, libwsmc), Cstring, ()))
    rc == WSMC_ENOTPD && throw(PosDefException(1))        # reference: cholesky in MvNormal(λΣ)
    error("libwsmc error $rc: $msg")
end

# ---------------------------------------------------------------------------------------
# the store (AbstractParticleStore, src/stores.jl:1-35)
# ---------------------------------------------------------------------------------------
mutable struct HipColumnStore <: WS.AbstractParticleStore
    ctx::Ptr{Cvoid}
    n::Int
    names::Vector{Symbol}
    ids::Dict{Symbol,Int32}
    dims::Dict{Symbol,Int}
    tmp::Int                       # counter for host-materialised temporaries
end

"""
    HipColumnStore(n; seed=42, device=0)
    HipColumnStore(n; gpus=8, devices=0:7, seed=42, transport=:rccl, shard_mode=:island)

One store of `n` particles on one device, or — `gpus > 1` — one handle over `gpus` devices
(`wsmc_create_multi`): contiguous shards, RCCL communicators from `ncclCommInitAll`, every
operator fanned out to the shards by the library, host vectors of all `n` particles split and
joined there. Julia stays single-threaded (src/types.jl:24-26) and needs no MPI launcher.
`shard_mode = :exact` resamples the whole population with the one-device bits.
"""
function HipColumnStore(n::Integer; seed::Integer=42, device::Integer=0, gpus::Integer=1,
                        devices=nothing, transport::Symbol=:rccl, shard_mode::Symbol=:island)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    if gpus == 1 && devices === nothing
        check(ccall((:wsmc_create, libwsmc), Cint, (Ptr{Ptr{Cvoid}}, Int64, Int32, UInt64),
                    h, n, device, seed % UInt64))
    else
        devs = Int32.(devices === nothing ? collect(0:gpus-1) : collect(devices))
        length(devs) == gpus || throw(ArgumentError("devices must list one device per shard"))
        tr = transport === :rccl ? Int32(0) : transport === :host ? Int32(1) :
             throw(ArgumentError("transport must be :rccl or :host"))
        check(ccall((:wsmc_create_multi, libwsmc), Cint,
                    (Ptr{Ptr{Cvoid}}, Int64, Int32, Ptr{Int32}, UInt64, Int32),
                    h, n, gpus, devs, seed % UInt64, tr))
        if shard_mode === :exact
            check(ccall((:wsmc_comm_set_shard_mode, libwsmc), Cint, (Ptr{Cvoid}, Int32), h[], 1))
        end
    end
    s = HipColumnStore(h[], Int(n), Symbol[], Dict{Symbol,Int32}(), Dict{Symbol,Int}(), 0)
    finalizer(s) do s
        s.ctx == C_NULL || ccall((:wsmc_destroy, libwsmc), Cint, (Ptr{Cvoid},), s.ctx)
        s.ctx = C_NULL
    end
    return s
end

nparticles(s::HipColumnStore) = s.n
hascol(s::HipColumnStore, name::Symbol) = haskey(s.ids, name)
colnames(s::HipColumnStore) = s.names

function column!(s::HipColumnStore, name::Symbol, dim::Integer)
    haskey(s.ids, name) && return s.ids[name]
    id = Ref{Int32}(0)
    check(ccall((:wsmc_col_create, libwsmc), Cint, (Ptr{Cvoid}, Cstring, Int32, Ptr{Int32}),
                s.ctx, String(name), dim, id))
    s.ids[name] = id[]
    s.dims[name] = dim
    push!(s.names, name)
    return id[]
end

"""
    lazy!(s, on)      materialize!(s)

The store's genealogy (DESIGN.md §3 "Lazy genealogy"): with `on` (the default) a Resample logs
its ancestors and columns catch up when read; `lazy!(s, false)` restores ColumnStore's eager
gather of every column at every resample (src/stores.jl:105-128). `materialize!` brings every
column up to date now (a `getcol` does it for its column anyway).
"""
lazy!(s::HipColumnStore, on::Bool) =
    check(ccall((:wsmc_store_set_lazy, libwsmc), Cint, (Ptr{Cvoid}, Int32), s.ctx, on ? 1 : 0))
materialize!(s::HipColumnStore) = check(ccall((:wsmc_store_materialize, libwsmc), Cint, (Ptr{Cvoid},), s.ctx))

"""Host copy of a column: `Vector{Float64}` (dim 1) or `Vector{Vector{Float64}}`."""
function download(s::HipColumnStore, name::Symbol)
    d = s.dims[name]
    buf = Vector{Float64}(undef, d * s.n)
    check(ccall((:wsmc_col_download, libwsmc), Cint, (Ptr{Cvoid}, Int32, Ptr{Float64}), s.ctx, s.ids[name], buf))
    d == 1 && return buf
    m = reshape(buf, s.n, d)                     # device layout is SoA [dim][N]
    return [m[i, :] for i in 1:s.n]
end

function upload!(s::HipColumnStore, name::Symbol, v::AbstractVector)
    d = eltype(v) <: AbstractVector ? length(first(v)) : 1
    id = column!(s, name, d)
    buf = d == 1 ? Vector{Float64}(v) : vec(permutedims(reduce(hcat, v)))   # -> [dim][N]
    check(ccall((:wsmc_col_upload, libwsmc), Cint, (Ptr{Cvoid}, Int32, Ptr{Float64}), s.ctx, id, buf))
end

"""The generic write path (src/stores.jl:85-96): evaluated on the host, then uploaded."""
function broadcast_setcol!(s::HipColumnStore, name::Symbol, f, args::Tuple)
    upload!(s, name, f.(map(materialize_host, args)...))
    return nothing
end

"""resample!(store, indices) with 1-based Julia indices (src/stores.jl:105-117)."""
function resample!(s::HipColumnStore, indices::AbstractVector{<:Integer})
    idx = Int32.(indices .- 1)
    check(ccall((:wsmc_store_resample, libwsmc), Cint, (Ptr{Cvoid}, Ptr{Int32}), s.ctx, idx))
    return nothing
end

# device proxies --------------------------------------------------------------------------
"""Component `comp` (0-based) of device column `id` — or the whole column when `comp < 0`."""
struct DeviceColumn <: AbstractVector{Float64}
    store::HipColumnStore
    name::Symbol
    comp::Int32
end
Base.size(c::DeviceColumn) = (c.store.n,)
Base.getindex(c::DeviceColumn, i::Int) = materialize_host(c)[i]   # generic host code: slow but correct

"""Lazy affine form c0 + Σ coef·col[comp] (≤ 2 terms: the wsmc_operand shape)."""
struct DeviceExpr
    store::HipColumnStore
    c0::Float64
    terms::Vector{Tuple{Symbol,Int32,Float64}}
end

getcol(s::HipColumnStore, name::Symbol) = DeviceColumn(s, name, s.dims[name] == 1 ? Int32(0) : Int32(-1))

struct DeviceStyle <: Broadcast.BroadcastStyle end
Base.BroadcastStyle(::Type{DeviceColumn}) = DeviceStyle()
Base.BroadcastStyle(::DeviceStyle, ::Broadcast.BroadcastStyle) = DeviceStyle()

lift(x::DeviceColumn) = DeviceExpr(x.store, 0.0, [(x.name, x.comp, 1.0)])
lift(x::DeviceExpr) = x
lift(x::Base.RefValue{<:Real}) = x[]
lift(x::Real) = x
lift(bc::Broadcast.Broadcasted) = affine(bc.f, map(lift, bc.args)...)

affine(::typeof(+), a::DeviceExpr, b::Real) = DeviceExpr(a.store, a.c0 + b, a.terms)
affine(::typeof(+), a::Real, b::DeviceExpr) = affine(+, b, a)
affine(::typeof(+), a::DeviceExpr, b::DeviceExpr) = DeviceExpr(a.store, a.c0 + b.c0, vcat(a.terms, b.terms))
affine(::typeof(-), a::DeviceExpr, b::Real) = DeviceExpr(a.store, a.c0 - b, a.terms)
affine(::typeof(-), a::Real, b::DeviceExpr) = affine(+, affine(*, -1.0, b), a)
affine(::typeof(-), a::DeviceExpr, b::DeviceExpr) = affine(+, a, affine(*, -1.0, b))
affine(::typeof(*), a::Real, b::DeviceExpr) = DeviceExpr(b.store, a * b.c0, [(n, c, a * k) for (n, c, k) in b.terms])
affine(::typeof(*), a::DeviceExpr, b::Real) = affine(*, b, a)
affine(::typeof(getindex), a::DeviceExpr, k::Integer) =                    # x[k] of a vector column
    DeviceExpr(a.store, a.c0, [(n, Int32(k - 1), coef) for (n, _, coef) in a.terms])
affine(f, args...) = nothing                                               # not affine: host path

# general expressions (wsmc_assign_expr, include/wsmc.h) ---------------------------------------
"""A fused broadcast as a postfix program (`wsmc_xinst`s) over device columns."""
struct DeviceProgram
    store::HipColumnStore
    ins::Vector{WsmcXInst}
end
const XOP1 = Dict{Any,Int32}(- => 2, abs => 3, sqrt => 4, exp => 5, log => 6, log1p => 7, sin => 8, cos => 9, (!) => 11)
const XOP2 = Dict{Any,Int32}(+ => 16, - => 17, * => 18, / => 19, min => 20, max => 21, (^) => 22, (<) => 23,
                             (<=) => 24, (>) => 25, (>=) => 26, (==) => 27, (!=) => 28, (&) => 29, (|) => 30)
xconst(v) = WsmcXInst(0, -1, 0, 0, Float64(v))
# postfix code of one broadcast argument, or nothing when something has no device form
function xcode(s::HipColumnStore, x)
    x isa Base.RefValue && x[] isa Real && return [xconst(x[])]
    x isa Real && return [xconst(x)]
    x isa DeviceColumn && return [WsmcXInst(1, s.ids[x.name], max(x.comp, 0), 0, 0.0)]
    x isa DeviceExpr && return xcode_affine(s, x)
    x isa Broadcast.Broadcasted || return nothing
    f, a = x.f, x.args
    if f === ifelse && length(a) == 3
        parts = map(y -> xcode(s, y), a)
        any(isnothing, parts) && return nothing
        return vcat(parts..., [WsmcXInst(31, -1, 0, 0, 0.0)])
    elseif f === (^) && length(a) == 2 && (a[2] isa Integer || (a[2] isa Base.RefValue && a[2][] isa Integer))
        n = a[2] isa Integer ? a[2] : a[2][]                       # x^n: literal_pow / pow_body
        b = xcode(s, a[1])
        return b === nothing ? nothing : vcat(b, [WsmcXInst(10, -1, 0, 0, Float64(n))])
    elseif f === Base.literal_pow && length(a) == 3                # x^2 lowered by the parser
        n = typeof(a[3] isa Base.RefValue ? a[3][] : a[3]).parameters[1]
        b = xcode(s, a[2])
        return b === nothing ? nothing : vcat(b, [WsmcXInst(10, -1, 0, 0, Float64(n))])
    elseif length(a) == 1 && haskey(XOP1, f)
        b = xcode(s, a[1])
        return b === nothing ? nothing : vcat(b, [WsmcXInst(XOP1[f], -1, 0, 0, 0.0)])
    elseif length(a) >= 2 && haskey(XOP2, f)                      # n-ary + and * fold left, as Julia's
        parts = map(y -> xcode(s, y), a)
        any(isnothing, parts) && return nothing
        code = parts[1]
        for p in parts[2:end]
            code = vcat(code, p, [WsmcXInst(XOP2[f], -1, 0, 0, 0.0)])
        end
        return code
    end
    return nothing
end
function xcode_affine(s::HipColumnStore, e::DeviceExpr)
    code = WsmcXInst[]
    for (k, (n, c, coef)) in enumerate(e.terms)
        t = coef == 1.0 ? [WsmcXInst(1, s.ids[n], max(c, 0), 0, 0.0)] :
            [xconst(coef), WsmcXInst(1, s.ids[n], max(c, 0), 0, 0.0), WsmcXInst(18, -1, 0, 0, 0.0)]
        code = k == 1 ? t : vcat(code, t, [WsmcXInst(16, -1, 0, 0, 0.0)])
    end
    isempty(code) && return [xconst(e.c0)]
    return e.c0 == 0.0 ? code : vcat(code, [xconst(e.c0), WsmcXInst(16, -1, 0, 0, 0.0)])
end
# the stack depth a program needs (the library refuses > 8 values, > 96 instructions)
function xdepth(ins)
    sp = 0; m = 0
    for i in ins
        sp += i.op <= 1 ? 1 : i.op <= 11 ? 0 : i.op == 31 ? -2 : -1
        m = max(m, sp)
    end
    return m
end
"""Evaluate a program on the device into column `id` (component 0) (wsmc_assign_expr)."""
function assign_program!(s::HipColumnStore, id::Int32, p::DeviceProgram)
    len = Int32[length(p.ins), 0, 0, 0]
    check(ccall((:wsmc_assign_expr, libwsmc), Cint, (Ptr{Cvoid}, Int32, Ptr{WsmcXInst}, Ptr{Int32}),
                s.ctx, id, p.ins, len))
end

function Broadcast.materialize(bc::Broadcast.Broadcasted{DeviceStyle})
    e = lift(bc)
    e isa DeviceExpr && length(e.terms) <= 2 && return e
    s = first(a.store for a in Broadcast.flatten(bc).args if a isa DeviceColumn)
    code = xcode(s, bc)
    code !== nothing && length(code) <= 96 && xdepth(code) <= 8 && return DeviceProgram(s, code)
    return Broadcast.materialize(Broadcast.broadcasted(bc.f, map(materialize_host, bc.args)...))
end

materialize_host(x) = x
materialize_host(c::DeviceColumn) =
    c.comp < 0 ? download(c.store, c.name) : getindex.(download(c.store, c.name), c.comp + 1)
materialize_host(e::DeviceExpr) = e.c0 .+ sum(k .* materialize_host(DeviceColumn(e.store, n, c)) for (n, c, k) in e.terms)

"""A `wsmc_operand` for one scalar argument; host vectors become temporary device columns."""
function operand(s::HipColumnStore, x)
    x isa Base.RefValue && return const_operand(x[])
    x isa Real && return const_operand(x)
    x isa DeviceColumn && (x = lift(x))
    if x isa DeviceProgram                        # a general argument: a temporary device column
        s.tmp += 1
        id = column!(s, Symbol("__wsmc_tmp", s.tmp), 1)
        assign_program!(s, id, x)
        return WsmcOperand(0.0, (id, Int32(-1)), (Int32(0), Int32(0)), (1.0, 0.0))
    end
    if x isa DeviceExpr
        cols = [(s.ids[n], c < 0 ? Int32(0) : c, k) for (n, c, k) in x.terms]
        pad = (Int32(-1), Int32(0), 0.0)
        a = length(cols) >= 1 ? cols[1] : pad
        b = length(cols) >= 2 ? cols[2] : pad
        return WsmcOperand(x.c0, (a[1], b[1]), (a[2], b[2]), (a[3], b[3]))
    end
    s.tmp += 1                                    # host-materialised argument
    name = Symbol("__wsmc_tmp", s.tmp)
    upload!(s, name, collect(Float64, x))
    return WsmcOperand(0.0, (s.ids[name], Int32(-1)), (Int32(0), Int32(0)), (1.0, 0.0))
end

"""Operands of a (possibly vector) argument, component by component."""
function operands(s::HipColumnStore, x, dim::Integer)
    if x isa Base.RefValue && x[] isa AbstractVector
        v = x[]
        return ntuple(k -> const_operand(k <= dim ? v[k] : 0.0), 4)
    elseif x isa DeviceColumn && x.comp < 0
        return ntuple(k -> operand(s, DeviceColumn(s, x.name, Int32(min(k, dim) - 1))), 4)
    end
    o = operand(s, x)
    return (o, o, o, o)
end

# kernels recognised by identity (src/default_kernels.jl:83-102) --------------------------
function device_dist(s::HipColumnStore, kernel, args)
    K = WS.default_kernels
    if kernel === K.Normal
        mu, sigma = args
        o = operand(s, mu)
        return WsmcDist(FAM_NORMAL, MEAN_AFFINE, 1, 0, (o, o, o, o), operand(s, sigma), (0.0, 0.0))
    elseif kernel === K.Uniform
        a, b = map(x -> x isa Base.RefValue ? x[] : x, args)
        z = const_operand(0.0)
        return WsmcDist(FAM_UNIFORM, MEAN_AFFINE, 1, 0, (z, z, z, z), const_operand(1.0), (Float64(a), Float64(b)))
    elseif kernel === K.MvNormal
        mu, Sigma = args
        S = Sigma isa Base.RefValue ? Sigma[] : Sigma
        d = size(S, 1)
        var = S[1, 1]
        S == var * I(d) &&
            return WsmcDist(FAM_MVNORMAL_ISO, MEAN_AFFINE, d, 0, operands(s, mu, d), const_operand(var), (0.0, 0.0))
        d <= 3 || return nothing                          # full covariance: dim <= 3
        # a full constant Σ: the library packs its Cholesky factor into the dist
        # (wsmc_dist_mvnormal_cov; PosDefException / non-symmetric Σ come back as errors)
        ops = operands(s, mu, d)
        z = const_operand(0.0)
        r = Ref(WsmcDist(FAM_MVNORMAL, MEAN_AFFINE, d, 0, ntuple(k -> k <= d ? ops[k] : z, 4), z, (0.0, 0.0)))
        Sm = Matrix{Float64}(transpose(Matrix{Float64}(S)))   # row-major for the C side
        check(ccall((:wsmc_dist_mvnormal_cov, libwsmc), Cint, (Ptr{WsmcDist}, Ptr{Float64}), r, Sm))
        return r[]
    end
    for (name, fam, li, si) in EXT_FAMILIES
        if hasproperty(K, name) && kernel === getproperty(K, name)
            loc = li == 0 ? const_operand(0.0) : operand(s, args[li])
            sc = si == 0 ? const_operand(1.0) : operand(s, args[si])
            return WsmcDist(Int32(fam), MEAN_AFFINE, 1, 0, (loc, loc, loc, loc), sc, (0.0, 0.0))
        end
    end
    return nothing
end

# ---------------------------------------------------------------------------------------
# operators on SMCState{<:HipColumnStore}
# ---------------------------------------------------------------------------------------
const HipState = SMCState{<:HipColumnStore}

function mirror_flags!(state::HipState)
    st = Ref{WsmcState}()
    check(ccall((:wsmc_get_state, libwsmc), Cint, (Ptr{Cvoid}, Ptr{WsmcState}), state.store.ctx, st))
    state.resampled = st[].resampled != 0
    state.weights_changed = st[].weights_changed != 0
    return st[]
end

function apply!(t::WS.Assign, state::HipState)
    s = state.store
    v = t.argfn(state)
    if v isa DeviceProgram                        # a general right-hand side: wsmc_assign_expr
        assign_program!(s, column!(s, t.lhs, 1), v)
        return WS.advance!(state)
    end
    d = v isa DeviceColumn && v.comp < 0 ? s.dims[v.name] : 1
    id = column!(s, t.lhs, d)
    ops = operands(s, v, d)
    check(ccall((:wsmc_assign, libwsmc), Cint, (Ptr{Cvoid}, Int32, Ptr{WsmcOperand}), s.ctx, id, Ref(ops)))
    WS.advance!(state)
end

"""
    importance_kernel(proposal, target)

`WeightedSampling.importance_kernel` (src/default_kernels.jl:69-73), registered so that a
`Sample` through it lowers to `wsmc_sample_importance` (draw from `proposal`, weights +=
logpdf(target) − logpdf(proposal), tape term = logpdf(target)). Kernels built by the
reference's own `importance_kernel` are recognised too, through the closures' captured
`proposal` / `target` fields.
"""
const IMPORTANCE = IdDict{Any,Tuple{Any,Any}}()
function importance_kernel(proposal, target)
    k = WS.importance_kernel(proposal, target)
    IMPORTANCE[k] = (proposal, target)
    return k
end
function importance_parts(k)
    haskey(IMPORTANCE, k) && return IMPORTANCE[k]
    f = k.weighter
    (hasfield(typeof(f), :proposal) && hasfield(typeof(f), :target)) || return nothing
    return (getfield(f, :proposal), getfield(f, :target))
end

"""A Distributions.jl object with constant parameters as a `WsmcDist` (or `nothing`)."""
function const_dist(d)
    z = const_operand(0.0)
    d isa Normal && return WsmcDist(FAM_NORMAL, MEAN_AFFINE, 1, 0, ntuple(_ -> const_operand(d.μ), 4),
                                    const_operand(d.σ), (0.0, 0.0))
    d isa Uniform && return WsmcDist(FAM_UNIFORM, MEAN_AFFINE, 1, 0, (z, z, z, z), const_operand(1.0), (d.a, d.b))
    return nothing
end

function apply!(t::WS.Sample, state::HipState)
    s = state.store
    args = t.argfn(state)
    if t.kernel.weighter !== nothing
        # A weighted Sample lowers only for importance kernels over device families. Any other
        # weighter would need the host to weigh AND extend the device's score tape and depth,
        # so it is refused rather than desynchronising weights_changed / depth from the
        # device (src/transformers.jl:172-182).
        parts = importance_parts(t.kernel)
        pd, td = parts === nothing ? (nothing, nothing) : map(const_dist, parts)
        (pd === nothing || td === nothing) &&
            error("WeightedSamplingHIP: weighted Sample kernel not supported on the device path " *
                  "(importance_kernel over constant Normal / Uniform is)")
        id = column!(s, t.lhs, 1)
        check(ccall((:wsmc_sample_importance, libwsmc), Cint, (Ptr{Cvoid}, Int32, Ref{WsmcDist}, Ref{WsmcDist}),
                    s.ctx, id, pd, td))
        state.weights_changed = true
        WS.advance!(state)
        return nothing
    end
    dist = device_dist(s, t.kernel, args)
    dist === nothing && error("WeightedSamplingHIP: Sample kernel not supported on the device path " *
                              "(Normal, Uniform, isotropic MvNormal and importance_kernel are)")
    id = column!(s, t.lhs, dist.dim)
    check(ccall((:wsmc_sample, libwsmc), Cint, (Ptr{Cvoid}, Int32, Ref{WsmcDist}), s.ctx, id, dist))
    WS.advance!(state)
end

for (T, fn) in ((WS.Observe, :wsmc_observe), (WS.Weight, :wsmc_weight))
    @eval function apply!(t::$T, state::HipState)
        s = state.store
        args = t.argfn(state)
        dist = device_dist(s, t.kernel, args)
        dist === nothing && error("WeightedSamplingHIP: kernel not supported on the device path")
        x = $(T === WS.Observe ? :(t.lhsfn(state)) : :(Ref(0.0)))
        check(ccall(($(QuoteNode(fn)), libwsmc), Cint, (Ptr{Cvoid}, Ref{WsmcDist}, Ptr{WsmcOperand}),
                    s.ctx, dist, Ref(operands(s, x, dist.dim))))
        state.weights_changed = true
        WS.advance!(state)
    end
end

function apply!(::WS.Resample, state::HipState)
    r = Ref{Int32}(0)
    e = Ref{Float64}(0.0)
    check(ccall((:wsmc_resample, libwsmc), Cint, (Ptr{Cvoid}, Float64, Int32, Ptr{Int32}, Ptr{Float64}),
                state.store.ctx, state.ess_perc_min, RESAMPLE_STRATIFIED, r, e))
    mirror_flags!(state)
    return nothing
end

"""`Move` with the built-in `RW` / `autoRW` proposals (recognised by identity)."""
# a Move's arguments: proposal kind, step, targets, bounds (src/move_kernels.jl:189-253)
function move_args(t::WS.Move, state::HipState)
    s = state.store
    args = t.argfn(state)
    kind = t.proposal === WS.autoRW ? PROPOSAL_AUTORW :
           t.proposal === WS.RW ? PROPOSAL_RW :
           error("WeightedSamplingHIP: only RW / autoRW proposals run on the device")
    step = isempty(args) ? 1e-3 : Float64(WS._scalar_arg(args[1]))
    bounds = length(args) >= 2 ? args[2] : nothing
    d = length(t.targets)
    ids = Int32[s.ids[c] for c in t.targets]
    lo = hi = nothing
    if bounds !== nothing
        b = WS._normalize_bounds(bounds, d)
        lo = Float64[x[1] for x in b]
        hi = Float64[x[2] for x in b]
    end
    return kind, step, ids, lo, hi
end

function apply!(t::WS.Move, state::HipState)
    kind, step, ids, lo, hi = move_args(t, state)
    div = t.diversity_threshold === nothing ? NaN : Float64(t.diversity_threshold)
    acc = Ref{Int64}(0)
    check(ccall((:wsmc_move, libwsmc), Cint,
                (Ptr{Cvoid}, Int32, Ptr{Int32}, Int32, Float64, Ptr{Float64}, Ptr{Float64}, Int32, Float64, Ptr{Int64}),
                state.store.ctx, kind, ids, length(ids), step, lo === nothing ? C_NULL : lo,
                hi === nothing ? C_NULL : hi, state.depth, div, acc))
    return nothing
end

# wsmc_move_spec (include/wsmc.h): one Move of a statement block
struct MoveSpec
    proposal::Int32
    d::Int32
    targets::NTuple{4,Int32}
    bounded::Int32
    target_depth::Int32
    step::Float64
    lo::NTuple{4,Float64}
    hi::NTuple{4,Float64}
end

# A Move's arguments do not read the state when its argfn gives the same arguments without one
# (`autoRW()`, `autoRW(1e-3, (0, Inf))`: the @model lowering's literal arguments); an argfn
# that reads the state (say a step from a column's spread) must see the state after the Moves
# before it, as the reference applies the steps in order (src/transformers.jl:331-334).
function state_free_args(m::WS.Move, state::HipState)
    try
        return m.argfn(nothing) == m.argfn(state)
    catch
        return false
    end
end

# A Sequence of Moves — the body of `if resampled ... end` (examples/linear_regression.jl:23-24)
# or a sweep — is one wsmc_move_block call: the sequential Moves' results, as one moments
# pass, one combine and one Move kernel when the block fuses (disjoint autoRW targets). Only
# when every Move's arguments are state-free and it has at most 4 targets; otherwise the
# steps run one by one, each argfn evaluated when its Move runs.
function apply!(t::WS.Sequence, state::HipState)
    steps = t.steps
    if !isempty(steps) && all(x -> x isa WS.Move && x.diversity_threshold === nothing &&
                                   length(x.targets) <= 4 && state_free_args(x, state), steps)
        specs = map(steps) do m
            kind, step, ids, lo, hi = move_args(m, state)
            d = length(ids)
            pad(v, x) = ntuple(k -> k <= d ? v[k] : x, 4)
            MoveSpec(kind, d, pad(ids, Int32(-1)), lo === nothing ? 0 : 1, state.depth, step,
                     lo === nothing ? ntuple(_ -> -Inf, 4) : pad(lo, -Inf),
                     hi === nothing ? ntuple(_ -> Inf, 4) : pad(hi, Inf))
        end
        v = collect(MoveSpec, specs)
        acc = zeros(Int64, length(v))
        check(ccall((:wsmc_move_block, libwsmc), Cint, (Ptr{Cvoid}, Int32, Ptr{MoveSpec}, Int32, Ptr{Int64}),
                    state.store.ctx, length(v), v, 0, acc))
        return nothing
    end
    foreach(step -> apply!(step, state), steps)
    return nothing
end

# weights live on the device; the host vector is a mirror refreshed on demand ------------
function sync_weights!(state::HipState)
    resize!(state.weights, state.store.n)
    check(ccall((:wsmc_weights_download, libwsmc), Cint, (Ptr{Cvoid}, Ptr{Float64}),
                state.store.ctx, state.weights))
    return state
end

function log_evidence(state::HipState)
    v = Ref{Float64}(0.0)
    check(ccall((:wsmc_log_evidence, libwsmc), Cint, (Ptr{Cvoid}, Ptr{Float64}), state.store.ctx, v))
    return v[]
end

const SPARK = ['▁', '▂', '▃', '▄', '▅', '▆', '▇', '█']

"""
    sample_device(state, n; replace=true) -> Dict{Symbol,Any}

`sample(state, n; replace)` (src/utils.jl:92-118): indices drawn and rows gathered on the
device; one entry per column (vector columns as a dim x n matrix).
"""
function sample_device(state::HipState, n::Integer; replace::Bool=true)
    s = state.store
    idx = zeros(Int64, n)
    check(ccall((:wsmc_sample_particles, libwsmc), Cint, (Ptr{Cvoid}, Int64, Int32, Ptr{Int64}),
                s.ctx, n, Int32(replace), idx))
    out = Dict{Symbol,Any}()
    for (name, id) in s.ids
        buf = Vector{Float64}(undef, s.dims[name] * n)
        check(ccall((:wsmc_col_gather_rows, libwsmc), Cint, (Ptr{Cvoid}, Int32, Ptr{Int64}, Int64, Ptr{Float64}),
                    s.ctx, id, idx, n, buf))
        out[name] = s.dims[name] == 1 ? buf : permutedims(reshape(buf, n, s.dims[name]))
    end
    return out
end

# multi-GPU: one process per GPU, each store a shard of one population (SURVEY §8(e)) ----
"""RCCL unique id, created on rank 0 and broadcast by the caller (e.g. `MPI.bcast`)."""
comm_unique_id() = (b = zeros(UInt8, 128); check(ccall((:wsmc_comm_unique_id, libwsmc), Cint, (Ptr{UInt8},), b)); b)

"""
    shard!(store, uid, world, rank, global_offset, global_n; exact=false)

Join the RCCL communicator as shard `rank` of `global_n` particles. `exact=true` makes
every Resample population-wide (`WSMC_SHARD_EXACT`: the single-GPU bits, particles move
between ranks); the default is island resampling (one record all-gather per step).
"""
function shard!(s::HipColumnStore, uid::Vector{UInt8}, world::Integer, rank::Integer, goff::Integer,
                gN::Integer; exact::Bool=false)
    check(ccall((:wsmc_comm_init, libwsmc), Cint, (Ptr{Cvoid}, Ptr{UInt8}, Int32, Int32, Int64, Int64),
                s.ctx, uid, world, rank, goff, gN))
    exact && check(ccall((:wsmc_comm_set_shard_mode, libwsmc), Cint, (Ptr{Cvoid}, Int32), s.ctx, 1))
    return s
end

# analysis reductions (src/utils.jl) on the device: no N-sized download ---------------------
"""
    expectation(state, x) -> Float64

`expectation(f, state)` / `@E` (src/utils.jl:11, :23-58) for an affine expression of particle
variables, e.g. `expectation(state, getcol(state.store, :α) .+ 2.0 .* getcol(state.store, :β))`.
Non-affine expressions go through `operand`'s host path (a temporary device column).
"""
function expectation(state::HipState, x)
    op = operand(state.store, x isa Broadcast.Broadcasted ? Broadcast.materialize(x) : x)
    m = Ref{Float64}(0.0)
    check(ccall((:wsmc_weighted_moments, libwsmc), Cint,
                (Ptr{Cvoid}, Ref{WsmcOperand}, Int32, Ptr{Float64}, Ptr{Float64}),
                state.store.ctx, op, 1, m, C_NULL))
    return m[]
end

"""
    describe_device(state; cols=colnames(state.store)) -> Vector{NamedTuple}

The numeric part of `describe(state)` (src/utils.jl:157-289): weighted mean and std
(`corrected=false`), min, max and ESS per column, component-wise for vector columns. The
weighted median and the sparkline need a sort / histogram pass: `describe(sync!(state))`
on the host gives those.
"""
function describe_device(state::HipState; cols=collect(keys(state.store.ids)))
    s = state.store
    essp = Ref{Float64}(0.0)
    check(ccall((:wsmc_ess, libwsmc), Cint, (Ptr{Cvoid}, Ptr{Float64}), s.ctx, essp))
    rows = NamedTuple[]
    for name in cols
        haskey(s.ids, name) || throw(ArgumentError("Column $name not found in store"))
        id, d = s.ids[name], s.dims[name]
        μ, σ, lo, hi, med = Float64[], Float64[], Float64[], Float64[], Float64[]
        for k in 0:d-1
            op = WsmcOperand(0.0, (id, Int32(-1)), (Int32(k), Int32(0)), (1.0, 0.0))
            m, v = Ref{Float64}(0.0), Ref{Float64}(0.0)
            check(ccall((:wsmc_weighted_moments, libwsmc), Cint,
                        (Ptr{Cvoid}, Ref{WsmcOperand}, Int32, Ptr{Float64}, Ptr{Float64}), s.ctx, op, 1, m, v))
            a, b = Ref{Float64}(0.0), Ref{Float64}(0.0)
            check(ccall((:wsmc_col_minmax, libwsmc), Cint, (Ptr{Cvoid}, Int32, Int32, Ptr{Float64}, Ptr{Float64}),
                        s.ctx, id, Int32(k), a, b))
            md = Ref{Float64}(0.0)
            check(ccall((:wsmc_weighted_median, libwsmc), Cint, (Ptr{Cvoid}, Int32, Int32, Ptr{Float64}),
                        s.ctx, id, Int32(k), md))
            push!(μ, m[]); push!(σ, sqrt(v[])); push!(lo, a[]); push!(hi, b[]); push!(med, md[])
        end
        hist = ""
        if d == 1
            lv = zeros(Int32, 8)
            check(ccall((:wsmc_histogram, libwsmc), Cint, (Ptr{Cvoid}, Int32, Int32, Ptr{Int32}), s.ctx, id, 0, lv))
            hist = join(SPARK[l] for l in lv)
        end
        pick(x) = d == 1 ? x[1] : x
        push!(rows, (variable=name, mean=pick(μ), median=pick(med), std=pick(σ), min=pick(lo), max=pick(hi),
                     hist=hist, ess=s.n * essp[]))
    end
    return rows
end

"""
    ssm2d_run!(state, obs; q_var=0.1, r_var=0.5, keep_history=true) -> log_evidence

The fused fast path: one HIP-graph launch for the whole `run!` of examples/2D_ssm.jl:7-17
on a fresh state (columns x_1..x_{T+1}, v, dv as the reference's store would hold them).
"""
function ssm2d_run!(state::HipState, obs::AbstractMatrix; x0=(0.0, 0.0), v0=(1.0, 0.0), q_var=0.1,
                    r_var=0.5, keep_history=true)
    T = size(obs, 1)
    o = Vector{Float64}(vec(permutedims(Float64.(obs))))          # row-major T x 2
    ev = Ref{Float64}(0.0)
    check(ccall((:wsmc_ssm2d_run, libwsmc), Cint,
                (Ptr{Cvoid}, Ptr{Float64}, Int32, Ptr{Float64}, Ptr{Float64}, Float64, Float64, Float64, Int32,
                 Int32, Ptr{Float64}),
                state.store.ctx, o, T, collect(Float64, x0), collect(Float64, v0), q_var, r_var,
                state.ess_perc_min, RESAMPLE_STRATIFIED, keep_history, ev))
    mirror_flags!(state)
    return ev[]
end

end # module
