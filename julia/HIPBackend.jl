# HIPBackend.jl — the reference-side binding a PartitionedArrays.jl (0.2.9)
# maintainer would add (INTEGRATION.md §2).  It plugs libpa_hip.so in behind
# the AbstractBackend / AbstractPData plugin API (src/Interfaces.jl:12, 50):
#
#   * `HIPBackend <: AbstractBackend`, `HIPData{T,N} <: AbstractPData{T,N}`:
#     SequentialBackend semantics (all parts in this process, i_am_main,
#     MAIN = 1) with part p on device devices[mod1(p, end)];
#   * a host/device mirror per part of every PVector and PSparseMatrix
#     (SURVEY.md §7 (i)): host arrays stay the parts the reference's generic
#     code sees; `map_parts` downloads the parts whose device copy is newer
#     before it runs a task and marks them host-newer after; the hot
#     operations upload host-newer parts, run on the device, and mark their
#     outputs device-newer — so a CG loop never touches host memory;
#   * specialisations of the hot path for PVector/PSparseMatrix over HIPData:
#     mul! (Interfaces.jl:2246), exchange!/assemble! of vectors (2071-2106)
#     and matrices (2375-2404), dot/norm/sum (1767, 1973-1992), copyto!/
#     copy!/fill!/rmul! (1649-1680, 1966), the CG broadcasts (1688-1765) and
#     IterativeSolvers.cg! (v0.9, test_fdm.jl:115), and the COO triplet
#     exchange assemble!(I, J, V, rows) (2406-2492);
#   * everything else (PRange, Exchanger, add_gids!, gather/scatter setup
#     collectives) runs unchanged on the host parts.
#
# Not executed in this repository (no Julia on the build image); the Python
# host package partitionedarrays.jl_amd/ drives the same C-ABI with ctypes and
# is what the tests run.  tests/test_julia_shim.py checks this file
# statically: every helper it calls is defined here, and every ccall names an
# entry point of include/pa_hip.h with its number of arguments.

module HIPBackends

using PartitionedArrays
using LinearAlgebra
using SparseArrays
using SparseMatricesCSR
import IterativeSolvers
import PartitionedArrays: get_part_ids, map_parts, i_am_main, get_backend, get_part, gather!,
  gather_all!, scatter, async_exchange!, async_assemble!, num_parts, prun_debug, PVector,
  PSparseMatrix, PRange, SequentialData, AbstractPData, AbstractBackend, Table, Exchanger, MAIN,
  num_lids, num_oids, num_hids, oids_are_equal, hids_are_equal

export HIPBackend, HIPData

const libpa = get(ENV, "PA_HIP_LIB", "libpa_hip.so")

# ---- errors (SURVEY.md §8b: int status + pa_last_error) --------------------
function check(rc::Cint)
  rc == 0 && return nothing
  msg = unsafe_string(ccall((:pa_last_error, libpa), Cstring, ()))
  error("libpa_hip: " * msg)
end

const PA_F32, PA_F64, PA_C64, PA_C128 = Cint(0), Cint(1), Cint(2), Cint(3)
dtype_code(::Type{Float32}) = PA_F32
dtype_code(::Type{Float64}) = PA_F64
dtype_code(::Type{ComplexF32}) = PA_C64
dtype_code(::Type{ComplexF64}) = PA_C128
const DeviceEltype = Union{Float32,Float64,ComplexF32,ComplexF64}

function device_count()
  n = Ref{Cint}(0)
  check(ccall((:pa_device_count, libpa), Cint, (Ref{Cint},), n))
  Int(n[])
end

# ---- backend, part contexts ------------------------------------------------
mutable struct PartCtx
  h::Ptr{Cvoid}
  device::Int
  part::Int
end

"""
    HIPBackend(devices=0:ndev-1; share_streams=true)

All parts in this process; part p on device devices[mod1(p, end)].  Parts
on one device share a stream pair (pa_ctx_create_shared) and run each mul!
phase as one grouped launch.  Contexts are created once per partition shape
and reused by every get_part_ids call (get_part_ids(a::AbstractPData) is
called by the generic code, e.g. PRange(parts, n)).
"""
mutable struct HIPBackend <: AbstractBackend
  devices::Vector{Int}
  share_streams::Bool
  ctxs::Dict{Any,Array{PartCtx}}
end
HIPBackend(devices=collect(0:(device_count() - 1)); share_streams::Bool=true) =
  HIPBackend(collect(Int, devices), share_streams, Dict{Any,Array{PartCtx}}())

function _contexts(b::HIPBackend, shape)
  get!(b.ctxs, shape) do
    np = prod(shape)
    isempty(b.devices) && error("HIPBackend: no HIP device visible")
    leader = Dict{Int,PartCtx}()
    cs = map(1:np) do p
      d = b.devices[mod1(p, length(b.devices))]
      h = Ref{Ptr{Cvoid}}(C_NULL)
      if b.share_streams && haskey(leader, d)
        check(ccall((:pa_ctx_create_shared, libpa), Cint, (Cint, Cint, Ptr{Cvoid}, Ref{Ptr{Cvoid}}),
                    p, np, leader[d].h, h))
      else
        check(ccall((:pa_ctx_create, libpa), Cint, (Cint, Cint, Cint, Ref{Ptr{Cvoid}}), d, p, np, h))
      end
      c = PartCtx(h[], d, p)
      haskey(leader, d) || (leader[d] = c)
      c
    end
    reshape(cs, shape)
  end
end

"""
    HIPData{T,N} <: AbstractPData{T,N}

The parts (host objects: part ids, index sets, host Vectors of PVector
values, SparseMatrixCSC of PSparseMatrix values, ...) plus the part contexts
of the backend.  Device copies hang off the host objects (mirror tables
below), so the parts are exactly what the reference's generic code expects.
"""
struct HIPData{T,N} <: AbstractPData{T,N}
  parts::Array{T,N}
  ctxs::Array{PartCtx,N}
  backend::HIPBackend
end

get_part_ids(b::HIPBackend, nparts::Integer) =
  HIPData(collect(1:nparts), _contexts(b, (nparts,)), b)
get_part_ids(b::HIPBackend, nparts::Tuple) =
  HIPData(collect(LinearIndices(nparts)), _contexts(b, nparts), b)
prun_debug(driver::Function, b::HIPBackend, nparts) = PartitionedArrays.prun(driver, b, nparts)

Base.size(a::HIPData) = size(a.parts)
get_backend(a::HIPData) = a.backend      # the stored backend: no device query, no new contexts
i_am_main(::HIPData) = true
get_part(a::HIPData, part::Integer) = a.parts[part]
get_part(a::HIPData) = get_part(a, MAIN)

# Base.iterate: as SequentialData (SequentialBackend.jl:26-50), so that
# `I, J, V = map_parts(...)` destructures
function Base.iterate(a::HIPData)
  next = map(iterate, a.parts)
  any(isnothing, next) && return nothing
  HIPData(map(first, next), a.ctxs, a.backend), HIPData(map(_second, next), a.ctxs, a.backend)
end
function Base.iterate(a::HIPData, state::HIPData)
  next = map(iterate, a.parts, state.parts)
  any(isnothing, next) && return nothing
  HIPData(map(first, next), a.ctxs, a.backend), HIPData(map(_second, next), a.ctxs, a.backend)
end
_second(a) = a[2]

# map_parts with host/device coherence: the parts of the arguments whose
# device copy is newer are downloaded first; after the task every mirrored
# part of the arguments is taken as modified on the host (the task may write
# any of them; the next hot operation uploads it again).
function map_parts(task, args::HIPData...)
  @assert length(args) > 0
  @assert all(a -> length(a.parts) == length(first(args).parts), args)
  for a in args
    foreach(sync_host!, a.parts)
  end
  parts_out = map(task, map(a -> a.parts, args)...)
  for a in args
    foreach(mark_host_newer!, a.parts)
  end
  HIPData(parts_out, first(args).ctxs, first(args).backend)
end

# host collectives of the setup phase (ids, ptrs, Tables): SequentialBackend's
# (SequentialBackend.jl:73-200) on the host parts
_seq(a::HIPData) = SequentialData(a.parts)
gather!(rcv::HIPData, snd::HIPData) = (gather!(_seq(rcv), _seq(snd)); rcv)
gather_all!(rcv::HIPData, snd::HIPData) = (gather_all!(_seq(rcv), _seq(snd)); rcv)
function scatter(snd::HIPData)
  s = scatter(_seq(snd))
  HIPData(s.parts, snd.ctxs, snd.backend)
end
function async_exchange!(data_rcv::HIPData, data_snd::HIPData, parts_rcv::HIPData,
                         parts_snd::HIPData, t_in::HIPData)
  t = async_exchange!(_seq(data_rcv), _seq(data_snd), _seq(parts_rcv), _seq(parts_snd), _seq(t_in))
  HIPData(t.parts, data_rcv.ctxs, data_rcv.backend)
end

# ---- device mirrors and handle caches ------------------------------------
# state: :host (host copy newer), :device (device copy newer), :both (equal)
mutable struct VecMirror
  h::Ptr{Cvoid}
  state::Symbol
end
mutable struct MatMirror
  h::Ptr{Cvoid}
  nnz::Int
  state::Symbol
end
function _free_vec(m::VecMirror)
  m.h == C_NULL || ccall((:pa_vec_destroy, libpa), Cint, (Ptr{Cvoid},), m.h)
  m.h = C_NULL
end
function _free_mat(m::MatMirror)
  m.h == C_NULL || ccall((:pa_mat_destroy, libpa), Cint, (Ptr{Cvoid},), m.h)
  m.h = C_NULL
end

# Mirror tables keyed by object identity (a content hash of a 16.7 M-value
# part per lookup would cost more than the SpMV): objectid(x) → (WeakRef(x),
# mirror).  An entry whose host object has been collected is stale: the next
# insertion sweeps stale entries and frees their device copies.
const VEC_MIRRORS = Dict{UInt,Tuple{WeakRef,VecMirror}}()  # host part Vector → its pa_vec
const MAT_MIRRORS = Dict{UInt,Tuple{WeakRef,MatMirror}}()  # host part SparseMatrixCSC → its pa_mat
const IDX_CACHE = IdDict{Any,Ptr{Cvoid}}()          # (index set, part, nlids) → pa_index
const XCHG_CACHE = IdDict{Any,Ptr{Cvoid}}()         # (exchanger, part) → pa_xchg
const GIDS_SET = Dict{Ptr{Cvoid},Bool}()          # pa_index handles with their gid table attached
const MXCHG_CACHE = IdDict{Any,Vector{Ptr{Cvoid}}}()  # (matrix exchanger, matrix values) → nz pa_xchg per part

function _mirror(tab, x)
  e = get(tab, objectid(x), nothing)
  (e === nothing || e[1].value !== x) ? nothing : e[2]
end
function _set_mirror!(tab, x, m, free)
  for (k, (w, old)) in collect(tab)   # sweep: host objects gone since the last insertion
    if w.value === nothing
      free(old)
      delete!(tab, k)
    end
  end
  e = get(tab, objectid(x), nothing)
  e === nothing || free(e[2])          # a stale entry under a reused id
  tab[objectid(x)] = (WeakRef(x), m)
  m
end

# download / mark: Vectors through their mirror, views through their parent,
# matrices through theirs; anything else has no device copy
sync_host!(x) = nothing
mark_host_newer!(x) = nothing
function sync_host!(x::Vector)
  m = _mirror(VEC_MIRRORS, x)
  if m !== nothing && m.state === :device
    check(ccall((:pa_vec_download, libpa), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Int64), m.h, x, length(x)))
    m.state = :both
  end
  nothing
end
function mark_host_newer!(x::Vector)
  m = _mirror(VEC_MIRRORS, x)
  m === nothing || (m.state = :host)
  nothing
end
sync_host!(x::SubArray) = sync_host!(parent(x))
mark_host_newer!(x::SubArray) = mark_host_newer!(parent(x))
function sync_host!(A::SparseMatrixCSC)
  m = _mirror(MAT_MIRRORS, A)
  if m !== nothing && m.state === :device
    check(ccall((:pa_mat_get_values, libpa), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), m.h, nonzeros(A)))
    m.state = :both
  end
  nothing
end
function mark_host_newer!(A::SparseMatrixCSC)
  m = _mirror(MAT_MIRRORS, A)
  m === nothing || (m.state = :host)
  nothing
end
function sync_host!(A::SparseMatrixCSR)
  m = _mirror(MAT_MIRRORS, A)
  if m !== nothing && m.state === :device
    check(ccall((:pa_mat_get_values, libpa), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), m.h, nonzeros(A)))
    m.state = :both
  end
  nothing
end
function mark_host_newer!(A::SparseMatrixCSR)
  m = _mirror(MAT_MIRRORS, A)
  m === nothing || (m.state = :host)
  nothing
end
sync_host!(A::PartitionedArrays.SubSparseMatrix) = sync_host!(A.parent)
mark_host_newer!(A::PartitionedArrays.SubSparseMatrix) = mark_host_newer!(A.parent)

function _vec_handle(ctx::PartCtx, x::Vector{T}) where {T<:DeviceEltype}
  m = _mirror(VEC_MIRRORS, x)
  if m === nothing
    out = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pa_vec_create, libpa), Cint, (Ptr{Cvoid}, Cint, Int64, Ref{Ptr{Cvoid}}),
                ctx.h, dtype_code(T), length(x), out))
    m = _set_mirror!(VEC_MIRRORS, x, VecMirror(out[], :host), _free_vec)
  end
  if m.state === :host
    check(ccall((:pa_vec_upload, libpa), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Int64), m.h, x, length(x)))
    m.state = :both
  end
  m.h
end

"""pa_vec handles of the parts of `v` (uploading host-newer parts)."""
dev_vec(v::PVector) = [_vec_handle(v.values.ctxs[i], v.values.parts[i]) for i in eachindex(v.values.parts)]

"""after a device operation wrote `v`: its device copy is the newer one."""
function mark_device_newer!(v::PVector)
  for x in v.values.parts
    m = _mirror(VEC_MIRRORS, x)
    m === nothing || (m.state = :device)
  end
  v
end

function _idx_handle(ctx::PartCtx, ids)
  key = (ids, ctx.part, num_lids(ids))  # add_gid! grows an index set: a new num_lids is a new handle
  get!(IDX_CACHE, key) do
    o = Int32.(collect(ids.oid_to_lid))
    h = Int32.(collect(ids.hid_to_lid))
    out = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pa_index_create, libpa), Cint,
                (Ptr{Cvoid}, Int64, Int64, Ptr{Int32}, Int64, Ptr{Int32}, Ref{Ptr{Cvoid}}),
                ctx.h, num_lids(ids), length(o), o, length(h), h, out))
    out[]
  end
end

"""pa_index handles of the index sets of `r` (IndexSets.jl:215-421)."""
dev_idx(r::PRange) = [_idx_handle(r.partition.ctxs[i], r.partition.parts[i]) for i in eachindex(r.partition.parts)]

function _xchg_handle(ctx::PartCtx, ex::Exchanger, i::Integer)
  get!(XCHG_CACHE, (ex, i)) do
    pr = Int32.(ex.parts_rcv.parts[i]); ps = Int32.(ex.parts_snd.parts[i])
    lr = ex.lids_rcv.parts[i]; ls = ex.lids_snd.parts[i]
    out = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pa_xchg_create, libpa), Cint,
                (Ptr{Cvoid}, Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int32},
                 Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ref{Ptr{Cvoid}}),
                ctx.h, length(pr), pr, Int32.(lr.ptrs), Int32.(lr.data),
                length(ps), ps, Int32.(ls.ptrs), Int32.(ls.data), out))
    out[]
  end
end

"""pa_xchg handles of the Exchanger of `r` (Interfaces.jl:698-713, verbatim)."""
dev_xchg(r::PRange) = [_xchg_handle(r.partition.ctxs[i], r.exchanger, i) for i in eachindex(r.partition.parts)]

function _mat_handle(ctx::PartCtx, A::SparseMatrixCSC{Tv}, rows_h::Ptr{Cvoid}, cols_h::Ptr{Cvoid}) where {Tv<:DeviceEltype}
  m = _mirror(MAT_MIRRORS, A)
  if m !== nothing && m.nnz != nnz(A)  # new pattern: rebuild
    _free_mat(m)
    m = nothing
  end
  if m === nothing
    colptr = Vector{Int64}(A.colptr); rowval = Vector{Int64}(A.rowval)
    out = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pa_mat_from_csc, libpa), Cint,
                (Ptr{Cvoid}, Cint, Cint, Int64, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Cvoid},
                 Ptr{Cvoid}, Ptr{Cvoid}, Ref{Ptr{Cvoid}}),
                ctx.h, dtype_code(Tv), 8, size(A, 1), size(A, 2), colptr, rowval, nonzeros(A),
                rows_h, cols_h, out))
    m = _set_mirror!(MAT_MIRRORS, A, MatMirror(out[], nnz(A), :both), _free_mat)
  elseif m.state === :host  # same pattern, new values (fillstored!, re-assembly)
    check(ccall((:pa_mat_set_values, libpa), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), m.h, nonzeros(A)))
    m.state = :both
  end
  m.h
end

# a SparseMatrixCSR{Bi} part (SparseUtils.jl:189-300): pa_mat_from_csr keeps
# the CSR's per-row order and scales each product by α, (v*x)*α (:247)
function _mat_handle(ctx::PartCtx, A::SparseMatrixCSR{Bi,Tv}, rows_h::Ptr{Cvoid}, cols_h::Ptr{Cvoid}) where {Bi,Tv<:DeviceEltype}
  m = _mirror(MAT_MIRRORS, A)
  if m !== nothing && m.nnz != nnz(A)  # new pattern: rebuild
    _free_mat(m)
    m = nothing
  end
  if m === nothing
    rowptr = Vector{Int64}(A.rowptr); colval = Vector{Int64}(A.colval)
    out = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pa_mat_from_csr, libpa), Cint,
                (Ptr{Cvoid}, Cint, Cint, Cint, Int64, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Cvoid},
                 Ptr{Cvoid}, Ptr{Cvoid}, Ref{Ptr{Cvoid}}),
                ctx.h, dtype_code(Tv), 8, Bi, size(A, 1), size(A, 2), rowptr, colval, nonzeros(A),
                rows_h, cols_h, out))
    m = _set_mirror!(MAT_MIRRORS, A, MatMirror(out[], nnz(A), :both), _free_mat)
  elseif m.state === :host
    check(ccall((:pa_mat_set_values, libpa), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), m.h, nonzeros(A)))
    m.state = :both
  end
  m.h
end

"""pa_mat handles of the parts of `a` (owned-row SELL, built once from the
local SparseMatrixCSC or SparseMatrixCSR; values re-uploaded when the host
copy is newer)."""
function dev_mat(a::PSparseMatrix)
  rh, ch = dev_idx(a.rows), dev_idx(a.cols)
  [_mat_handle(a.values.ctxs[i], a.values.parts[i], rh[i], ch[i]) for i in eachindex(a.values.parts)]
end

function mark_device_newer!(a::PSparseMatrix)
  for A in a.values.parts
    m = _mirror(MAT_MIRRORS, A)
    m === nothing || (m.state = :device)
  end
  a
end

"""pa_xchg handles of the matrix exchanger of `a` (Interfaces.jl:2300-2372;
lids are CSC nz ids, Int64 as Table{Int})."""
function dev_mat_xchg(a::PSparseMatrix)
  A = dev_mat(a)
  get!(MXCHG_CACHE, (a.exchanger, a.values)) do
    ex = a.exchanger
    map(eachindex(a.values.parts)) do i
      pr = Int32.(ex.parts_rcv.parts[i]); ps = Int32.(ex.parts_snd.parts[i])
      lr = ex.lids_rcv.parts[i]; ls = ex.lids_snd.parts[i]
      out = Ref{Ptr{Cvoid}}(C_NULL)
      check(ccall((:pa_mat_xchg_create, libpa), Cint,
                  (Ptr{Cvoid}, Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int64},
                   Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int64}, Ref{Ptr{Cvoid}}),
                  A[i], length(pr), pr, Int32.(lr.ptrs), Int64.(lr.data),
                  length(ps), ps, Int32.(ls.ptrs), Int64.(ls.data), out))
      out[]
    end
  end
end

const HIPVector{T} = PVector{T,<:HIPData}
const HIPMatrix{T} = PSparseMatrix{T,<:HIPData}

# the tasks async operations hand back: the device work is already enqueued
# (stream-ordered); waiting on a task synchronises its part's streams
function _done_tasks(a::HIPData)
  tasks = map(a.ctxs) do c
    @task check(ccall((:pa_ctx_sync, libpa), Cint, (Ptr{Cvoid},), c.h))
  end
  HIPData(tasks, a.ctxs, a.backend)
end
function _wait_all(t0::AbstractPData)
  map_parts(t0) do t
    istaskstarted(t) || schedule(t)
    wait(t)
  end
  nothing
end

# ---- hot path: mul!(c, a, b, α, β) (Interfaces.jl:2246-2275) --------------
function LinearAlgebra.mul!(c::HIPVector{T}, a::HIPMatrix{T}, b::HIPVector{T}, α::Number, β::Number) where {T<:DeviceEltype}
  @assert oids_are_equal(c.rows, a.rows)
  @assert oids_are_equal(a.cols, b.rows)
  @assert hids_are_equal(a.cols, b.rows)
  A, yv, yi = dev_mat(a), dev_vec(c), dev_idx(c.rows)
  xv, xi, xg = dev_vec(b), dev_idx(b.rows), dev_xchg(b.rows)
  al = Ref{T}(T(α)); be = Ref{T}(T(β))
  check(ccall((:pa_spmv_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}},
               Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ref{T}, Ref{T}),
              length(A), A, yv, yi, xv, xi, xg, al, be))
  mark_device_newer!(c)
  mark_device_newer!(b)   # exchange!(b): its ghost values were replaced on the device
  c
end
LinearAlgebra.mul!(c::HIPVector{T}, a::HIPMatrix{T}, b::HIPVector{T}) where {T<:DeviceEltype} =
  mul!(c, a, b, one(T), zero(T))
function Base.:*(a::HIPMatrix{Ta}, b::HIPVector{Tb}) where {Ta,Tb}   # Interfaces.jl:2605-2610
  T = typeof(zero(Ta) * zero(Tb) + zero(Ta) * zero(Tb))
  c = PVector{T}(undef, a.rows)
  mul!(c, a, b)
end

# ---- exchange!/assemble! (Interfaces.jl:2071-2106, 2375-2404) --------------
function _exchange_all(v::HIPVector, op::Integer, rev::Integer, zero_ghosts::Integer)
  vv, vi, xg = dev_vec(v), dev_idx(v.rows), dev_xchg(v.rows)
  check(ccall((:pa_exchange_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Cint, Cint, Cint),
              length(vv), vv, xg, vi, op, rev, zero_ghosts))
  mark_device_newer!(v)
end
function async_exchange!(a::HIPVector{T}, t0::AbstractPData=PartitionedArrays._empty_tasks(a.rows.exchanger.parts_rcv)) where {T<:DeviceEltype}
  _wait_all(t0)
  _exchange_all(a, 0, 0, 0)
  _done_tasks(a.values)
end
function async_assemble!(a::HIPVector{T}, t0::AbstractPData=PartitionedArrays._empty_tasks(a.rows.exchanger.parts_rcv)) where {T<:DeviceEltype}
  async_assemble!(+, a, t0)
end
function async_assemble!(::typeof(+), a::HIPVector{T}, t0::AbstractPData=PartitionedArrays._empty_tasks(a.rows.exchanger.parts_rcv)) where {T<:DeviceEltype}
  _wait_all(t0)
  _exchange_all(a, 1, 1, 1)   # reverse(exchanger), +, then ghost values = 0
  _done_tasks(a.values)
end

function _mat_exchange_all(a::HIPMatrix, op::Integer, rev::Integer, zero_sent::Integer)
  A, mx = dev_mat(a), dev_mat_xchg(a)
  check(ccall((:pa_mat_exchange_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Cint, Cint, Cint), length(A), A, mx, op, rev, zero_sent))
  mark_device_newer!(a)
end
function async_exchange!(a::HIPMatrix{T}, t0::AbstractPData=PartitionedArrays._empty_tasks(a.exchanger.parts_rcv)) where {T<:DeviceEltype}
  _wait_all(t0)
  _mat_exchange_all(a, 0, 0, 0)
  _done_tasks(a.values)
end
function async_assemble!(::typeof(+), a::HIPMatrix{T}, t0::AbstractPData=PartitionedArrays._empty_tasks(a.exchanger.parts_rcv)) where {T<:DeviceEltype}
  _wait_all(t0)
  _mat_exchange_all(a, 1, 1, 1)
  _done_tasks(a.values)
end
async_assemble!(a::HIPMatrix{T}, t0::AbstractPData=PartitionedArrays._empty_tasks(a.exchanger.parts_rcv)) where {T<:DeviceEltype} =
  async_assemble!(+, a, t0)

# fillstored!(a, v) (Interfaces.jl:2127-2132) on the device copies; the host
# parts are refreshed on their next generic use (sync_host!)
function LinearAlgebra.fillstored!(a::HIPMatrix{T}, v) where {T<:DeviceEltype}
  A = dev_mat(a)
  s = Ref{T}(convert(T, v))
  for h in A
    check(ccall((:pa_mat_fillstored, libpa), Cint, (Ptr{Cvoid}, Ptr{T}), h, s))
  end
  mark_device_newer!(a)
  a
end

# ---- assemble!(I, J, V, rows) (Interfaces.jl:2406-2492) --------------------
# the triplets go to the device (pa_coo), the ghost rows' triplets move to
# their owners there (pa_coo_assemble_all: device copies / RCCL), and the
# assembled lists come back into I, J, V (resize!, as the reference does)
function _idx_gids_handle(ctx::PartCtx, ids)
  h = _idx_handle(ctx, ids)
  get!(GIDS_SET, h) do
    g = Int64.(collect(ids.lid_to_gid))
    check(ccall((:pa_index_set_gids, libpa), Cint, (Ptr{Cvoid}, Ptr{Int64}), h, g))
    true
  end
  h
end
function async_assemble!(I::HIPData{<:Vector{<:Integer}}, J::HIPData{<:Vector{<:Integer}},
                         V::HIPData{<:Vector{T}}, rows::PRange,
                         t0::AbstractPData=PartitionedArrays._empty_tasks(rows.exchanger.parts_rcv)) where {T<:DeviceEltype}
  _wait_all(t0)
  n = length(I.parts)
  coo = Vector{Ptr{Cvoid}}(undef, n)
  for i in 1:n
    out = Ref{Ptr{Cvoid}}(C_NULL)
    gi = Int64.(I.parts[i]); gj = Int64.(J.parts[i])
    check(ccall((:pa_coo_create, libpa), Cint,
                (Ptr{Cvoid}, Cint, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{T}, Ref{Ptr{Cvoid}}),
                I.ctxs[i].h, dtype_code(T), length(gi), gi, gj, V.parts[i], out))
    coo[i] = out[]
  end
  try
    ri = [_idx_gids_handle(rows.partition.ctxs[i], rows.partition.parts[i]) for i in 1:n]
    check(ccall((:pa_coo_assemble_all, libpa), Cint,
                (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}), n, coo, ri, dev_xchg(rows)))
    for i in 1:n
      m = Ref{Int64}(0)
      check(ccall((:pa_coo_size, libpa), Cint, (Ptr{Cvoid}, Ref{Int64}), coo[i], m))
      gi = Vector{Int64}(undef, m[]); gj = Vector{Int64}(undef, m[])
      resize!(V.parts[i], m[])
      check(ccall((:pa_coo_download, libpa), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Ptr{T}),
                  coo[i], gi, gj, V.parts[i]))
      resize!(I.parts[i], m[]); I.parts[i] .= gi
      resize!(J.parts[i], m[]); J.parts[i] .= gj
    end
  finally
    foreach(h -> ccall((:pa_coo_destroy, libpa), Cint, (Ptr{Cvoid},), h), coo)
  end
  _done_tasks(I)
end

# ---- reductions (Interfaces.jl:221-238, 1767-1772, 1973-1992) -------------
function LinearAlgebra.dot(a::HIPVector{T}, b::HIPVector{T}) where {T<:DeviceEltype}
  r = Ref{T}(zero(T))
  check(ccall((:pa_dot_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ref{T}),
              num_parts(a.values), dev_vec(a), dev_idx(a.rows), dev_vec(b), dev_idx(b.rows), r))
  r[]
end
function LinearAlgebra.norm(a::HIPVector{T}, p::Real=2) where {T<:DeviceEltype}
  p == 2 || return invoke(norm, Tuple{PVector,Real}, a, p)
  r = Ref{Float64}(0.0)
  check(ccall((:pa_norm2_all, libpa), Cint, (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ref{Float64}),
              num_parts(a.values), dev_vec(a), dev_idx(a.rows), r))
  r[]
end
function Base.sum(a::HIPVector{T}) where {T<:DeviceEltype}
  r = Ref{T}(zero(T))
  check(ccall((:pa_sum_all, libpa), Cint, (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ref{T}),
              num_parts(a.values), dev_vec(a), dev_idx(a.rows), r))
  r[]
end

# ---- vector updates (Interfaces.jl:1649-1680, 1688-1765, 1966-1971) -------
function Base.fill!(a::HIPVector{T}, v) where {T<:DeviceEltype}
  s = Ref{T}(T(v))
  for (h, x) in zip(dev_vec_nocopy(a), a.values.parts)
    check(ccall((:pa_vec_fill, libpa), Cint, (Ptr{Cvoid}, Ref{T}), h, s))
  end
  mark_device_newer!(a)
end
# a vector about to be overwritten everywhere: its host values need not be uploaded
function dev_vec_nocopy(v::PVector)
  map(eachindex(v.values.parts)) do i
    x = v.values.parts[i]
    m = _mirror(VEC_MIRRORS, x)
    if m === nothing
      m = _vec_handle_uninit(v.values.ctxs[i], x)
    elseif m.state === :host
      m.state = :both   # about to be overwritten on the device: no upload
    end
    m.h
  end
end
function _vec_handle_uninit(ctx::PartCtx, x::Vector{T}) where {T<:DeviceEltype}
  out = Ref{Ptr{Cvoid}}(C_NULL)
  check(ccall((:pa_vec_create, libpa), Cint, (Ptr{Cvoid}, Cint, Int64, Ref{Ptr{Cvoid}}),
              ctx.h, dtype_code(T), length(x), out))
  _set_mirror!(VEC_MIRRORS, x, VecMirror(out[], :both), _free_vec)
end

function Base.copyto!(a::HIPVector{T}, b::HIPVector{T}) where {T<:DeviceEltype}
  @assert oids_are_equal(a.rows, b.rows)
  same = a.rows.partition === b.rows.partition
  src = dev_vec(b)
  dst = same ? dev_vec_nocopy(a) : dev_vec(a)
  ia, ib = dev_idx(a.rows), dev_idx(b.rows)
  for i in eachindex(dst)
    check(ccall((:pa_vec_copy, libpa), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint),
                dst[i], ia[i], src[i], ib[i], same ? 1 : 0))
  end
  mark_device_newer!(a)
end
Base.copy!(a::HIPVector{T}, b::HIPVector{T}) where {T<:DeviceEltype} = copyto!(a, b)

# the scalar as Julia's broadcast types it: a Float64 (Real * Complex
# componentwise) or a ComplexF64 that widens T is passed as such and the
# elements are evaluated in Float64 / ComplexF64 (PA_BCAST_F64 / _C128);
# anything else is converted to T
const PA_BCAST_F64, PA_BCAST_C128 = Cint(8), Cint(16)
_bcast_scalar(::Type{T}, a::Float64) where {T} = (Ref{Float64}(a), PA_BCAST_F64)
_bcast_scalar(::Type{T}, a::ComplexF64) where {T<:Complex} = (Ref{ComplexF64}(a), PA_BCAST_C128)
_bcast_scalar(::Type{T}, a) where {T} = (Ref{T}(T(a)), Cint(0))

function _axpby!(y::HIPVector{T}, x::Union{Nothing,HIPVector{T}}, a, mode::Integer) where {T<:DeviceEltype}
  all_lids = x === nothing || y.rows === x.rows
  x === nothing || all_lids || @assert oids_are_equal(y.rows, x.rows)
  s, kind = _bcast_scalar(T, a)
  yv, xv, iy = dev_vec(y), (x === nothing ? fill(C_NULL, num_parts(y.values)) : dev_vec(x)), dev_idx(y.rows)
  for i in eachindex(yv)
    check(ccall((:pa_vec_axpby, libpa), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Cint),
                yv[i], xv[i], iy[i], s, Cint(mode) | kind, all_lids ? 1 : 0))
  end
  mark_device_newer!(y)
end
LinearAlgebra.rmul!(a::HIPVector{T}, v::Number) where {T<:DeviceEltype} = _axpby!(a, nothing, v, 4)

# Broadcasts: a lazy tree over HIP vectors; materialize! runs the patterns of
# the CG recurrence on the device (pa_vec_axpby modes 0-3, copies) and any
# other expression through the reference's host broadcast on synced parts.
struct HIPBroadcasted{F,A}
  f::F
  args::A
  rows::PRange
end
const HIPArg = Union{HIPVector,HIPBroadcasted}
_rows(a::HIPVector) = a.rows
_rows(a::HIPBroadcasted) = a.rows
Base.broadcasted(f, args::HIPArg...) = HIPBroadcasted(f, args, _rows(first(args)))
Base.broadcasted(f, a::Number, b::HIPArg) = HIPBroadcasted(f, (a, b), _rows(b))
Base.broadcasted(f, a::HIPArg, b::Number) = HIPBroadcasted(f, (a, b), _rows(a))

_scaled(b) = nothing
function _scaled(b::HIPBroadcasted)   # β .* u or u .* β
  b.f === (*) && length(b.args) == 2 || return nothing
  a1, a2 = b.args
  a1 isa Number && a2 isa HIPVector && return (a1, a2)
  a1 isa HIPVector && a2 isa Number && return (a2, a1)
  nothing
end

# (mode, x, scalar) of y .= expression, or nothing
function _axpby_pattern(y::HIPVector, bc::HIPBroadcasted)
  length(bc.args) == 2 || return (bc.f === identity && length(bc.args) == 1 && bc.args[1] isa HIPVector) ?
                                 (:copy, bc.args[1], nothing) : nothing
  a1, a2 = bc.args
  if bc.f === (+)
    s = _scaled(a2)
    s !== nothing && a1 isa HIPVector && s[2] === y && return (0, a1, s[1])   # u .= r .+ β.*u
    s !== nothing && a1 === y && return (1, s[2], s[1])                         # x .+= α.*u
  elseif bc.f === (-)
    s = _scaled(a2)
    s !== nothing && a1 === y && return (2, s[2], s[1])                         # r .-= α.*c
    a1 === y && a2 isa HIPVector && return (3, a2, nothing)                      # r .-= c
  end
  nothing
end

function Base.materialize!(y::HIPVector{T}, bc::HIPBroadcasted) where {T<:DeviceEltype}
  pat = _axpby_pattern(y, bc)
  # device patterns over vectors of y's partition (all lids, as the
  # reference's materialize! does when every argument shares y.rows)
  if pat !== nothing && (pat[2] isa HIPVector{T}) && pat[2].rows === y.rows
    mode, x, a = pat
    mode === :copy && return copyto!(y, x)
    return _axpby!(y, x, a === nothing ? zero(T) : a, mode)
  end
  # any other expression: the reference's host broadcast (Interfaces.jl:1688-1765)
  host = _host_broadcasted(bc)
  invoke(Base.materialize!, Tuple{PVector,PartitionedArrays.DistributedBroadcasted}, y, host)
end
Base.materialize!(y::PVector, bc::HIPBroadcasted) =
  invoke(Base.materialize!, Tuple{PVector,PartitionedArrays.DistributedBroadcasted}, y, _host_broadcasted(bc))
Base.materialize(bc::HIPBroadcasted) = Base.materialize(_host_broadcasted(bc))

_host_arg(a) = a
_host_arg(a::HIPBroadcasted) = _host_broadcasted(a)
function _host_broadcasted(bc::HIPBroadcasted)
  args = map(_host_arg, bc.args)
  # the generic methods (map_parts syncs the parts that are newer on the device)
  if length(args) == 2 && args[1] isa Number
    invoke(Base.broadcasted, Tuple{Any,Number,Union{PVector,PartitionedArrays.DistributedBroadcasted}}, bc.f, args...)
  elseif length(args) == 2 && args[2] isa Number
    invoke(Base.broadcasted, Tuple{Any,Union{PVector,PartitionedArrays.DistributedBroadcasted},Number}, bc.f, args...)
  else
    invoke(Base.broadcasted, Tuple{Any,Vararg{Union{PVector,PartitionedArrays.DistributedBroadcasted}}}, bc.f, args...)
  end
end

# ---- IterativeSolvers.cg! (v0.9) with the recurrence on the device --------
# (pa_cg_solve_all: the same iterates as the generic cg! over the
# specialisations above, bit for bit, with no host round trip per iteration)
# log = true returns IterativeSolvers' ConvergenceHistory: that keeps the
# generic cg! (over the specialisations above); verbose is not printed here.
function IterativeSolvers.cg!(x::HIPVector{T}, A::HIPMatrix{T}, b::HIPVector{T};
                              abstol::Real=zero(real(T)), reltol::Real=sqrt(eps(real(T))),
                              maxiter::Int=size(A, 2), log::Bool=false, initially_zero::Bool=false,
                              kwargs...) where {T<:DeviceEltype}
  if log || haskey(kwargs, :Pl) || haskey(kwargs, :statevars)
    return invoke(IterativeSolvers.cg!, Tuple{Any,Any,Any}, x, A, b; abstol=abstol, reltol=reltol,
                  maxiter=maxiter, log=log, initially_zero=initially_zero, kwargs...)
  end
  u, r, c = similar(x), similar(x), similar(x)
  bb = b.rows === x.rows ? b : copyto!(similar(x), b)
  its = Ref{Int64}(0); res = Ref{Float64}(0.0)
  check(ccall((:pa_cg_solve_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}},
               Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}},
               Float64, Float64, Int64, Cint, Ref{Int64}, Ref{Float64}, Ptr{Float64}),
              num_parts(x.values), dev_mat(A), dev_vec(x), dev_vec(bb), dev_vec_nocopy(u),
              dev_vec_nocopy(r), dev_vec_nocopy(c), dev_idx(x.rows), dev_xchg(x.rows),
              Float64(reltol), Float64(abstol), maxiter, Cint(16), its, res, Ptr{Float64}(C_NULL)))
  mark_device_newer!(x)
  x
end

end # module
