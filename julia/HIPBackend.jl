# HIPBackend.jl — the reference-side binding a PartitionedArrays.jl maintainer
# would add (see INTEGRATION.md).  It plugs libpa_hip.so in behind the
# AbstractBackend / AbstractPData plugin API (src/Interfaces.jl:12, 50) and
# specialises the hot path for PVector/PSparseMatrix whose parts are HIP parts.
# Not executed in this repository (no Julia on the build image); the Python
# host package partitionedarrays.jl_amd/ drives the same C-ABI with ctypes and
# is what the tests run.

module HIPBackends

using PartitionedArrays
using LinearAlgebra
using SparseArrays
import PartitionedArrays: get_part_ids, map_parts, i_am_main, get_backend, get_part,
  gather!, gather_all!, scatter, async_exchange!, prun, num_parts

const libpa = get(ENV, "PA_HIP_LIB", "libpa_hip.so")

# ---- errors ---------------------------------------------------------------
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

# ---- backend and partitioned data: SequentialBackend semantics, HIP parts --
struct HIPBackend <: AbstractBackend
  devices::Vector{Int}
end
HIPBackend() = HIPBackend(collect(0:(_device_count()-1)))

function _device_count()
  n = Ref{Cint}(0)
  check(ccall((:pa_device_count, libpa), Cint, (Ref{Cint},), n))
  Int(n[])
end

mutable struct PartCtx
  h::Ptr{Cvoid}
end

struct HIPData{T,N} <: AbstractPData{T,N}
  parts::Array{T,N}
  ctxs::Array{PartCtx,N}
end
Base.size(a::HIPData) = size(a.parts)
get_backend(a::HIPData) = HIPBackend()
i_am_main(::HIPData) = true
get_part(a::HIPData, part::Integer) = a.parts[part]
get_part(a::HIPData) = a.parts[PartitionedArrays.MAIN]

function _ctxs(b::HIPBackend, np::Integer)
  map(1:np) do p
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pa_ctx_create, libpa), Cint, (Cint, Cint, Cint, Ref{Ptr{Cvoid}}),
                b.devices[mod1(p, length(b.devices))], p, np, h))
    PartCtx(h[])
  end
end
get_part_ids(b::HIPBackend, nparts::Integer) = HIPData(collect(1:nparts), _ctxs(b, nparts))
function get_part_ids(b::HIPBackend, nparts::Tuple)
  parts = collect(LinearIndices(nparts))
  HIPData(parts, reshape(_ctxs(b, prod(nparts)), nparts))
end
function map_parts(task, args::HIPData...)
  parts_out = map(task, map(a -> a.parts, args)...)
  HIPData(parts_out, first(args).ctxs)
end
# gather!/gather_all!/scatter/async_exchange! on host data (setup only):
# identical to SequentialBackend.jl:73-200 — delegated.
for f in (:gather!, :gather_all!)
  @eval $f(rcv::HIPData, snd::HIPData) =
    (PartitionedArrays.$f(SequentialData(rcv.parts), SequentialData(snd.parts)); rcv)
end
scatter(snd::HIPData) = (s = scatter(SequentialData(snd.parts)); HIPData(s.parts, snd.ctxs))
function async_exchange!(data_rcv::HIPData, data_snd::HIPData, parts_rcv::HIPData,
                         parts_snd::HIPData, t_in::HIPData)
  t = async_exchange!(SequentialData(data_rcv.parts), SequentialData(data_snd.parts),
                      SequentialData(parts_rcv.parts), SequentialData(parts_snd.parts),
                      SequentialData(t_in.parts))
  HIPData(t.parts, data_rcv.ctxs)
end

# ---- device handles (created once per index set / exchanger / matrix) -------
function pa_index(ctx::PartCtx, ids::PartitionedArrays.AbstractIndexSet)
  o = Int32.(collect(ids.oid_to_lid)); h = Int32.(collect(ids.hid_to_lid))
  out = Ref{Ptr{Cvoid}}(C_NULL)
  check(ccall((:pa_index_create, libpa), Cint,
              (Ptr{Cvoid}, Int64, Int64, Ptr{Int32}, Int64, Ptr{Int32}, Ref{Ptr{Cvoid}}),
              ctx.h, num_lids(ids), length(o), o, length(h), h, out))
  out[]
end

function pa_xchg(ctx::PartCtx, parts_rcv, lids_rcv, parts_snd, lids_snd)
  pr = Int32.(parts_rcv); ps = Int32.(parts_snd)
  out = Ref{Ptr{Cvoid}}(C_NULL)
  check(ccall((:pa_xchg_create, libpa), Cint,
              (Ptr{Cvoid}, Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int32},
               Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ref{Ptr{Cvoid}}),
              ctx.h, length(pr), pr, lids_rcv.ptrs, Int32.(lids_rcv.data),
              length(ps), ps, lids_snd.ptrs, Int32.(lids_snd.data), out))
  out[]
end

function pa_mat(ctx::PartCtx, A::SparseMatrixCSC{Tv,Int64}, rows_h, cols_h) where Tv
  out = Ref{Ptr{Cvoid}}(C_NULL)
  check(ccall((:pa_mat_from_csc, libpa), Cint,
              (Ptr{Cvoid}, Cint, Cint, Int64, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Tv},
               Ptr{Cvoid}, Ptr{Cvoid}, Ref{Ptr{Cvoid}}),
              ctx.h, dtype_code(Tv), 8, size(A, 1), size(A, 2),
              A.colptr, A.rowval, A.nzval, rows_h, cols_h, out))
  out[]
end

# A device mirror per PVector part (values uploaded once, kept resident).
mutable struct DeviceVec{T}
  h::Ptr{Cvoid}
end
function DeviceVec(ctx::PartCtx, v::Vector{T}) where T
  out = Ref{Ptr{Cvoid}}(C_NULL)
  check(ccall((:pa_vec_create, libpa), Cint, (Ptr{Cvoid}, Cint, Int64, Ref{Ptr{Cvoid}}),
              ctx.h, dtype_code(T), length(v), out))
  check(ccall((:pa_vec_upload, libpa), Cint, (Ptr{Cvoid}, Ptr{T}, Int64), out[], v, length(v)))
  DeviceVec{T}(out[])
end

# ---- hot path: mul!(c, a, b, α, β) (Interfaces.jl:2246-2275) --------------
# `dev(x)` returns (pa_vec handles, pa_index handles, pa_xchg handles) cached
# on the objects; see INTEGRATION.md for the cache and coherence rules.
function LinearAlgebra.mul!(c::PVector{T,<:HIPData}, a::PSparseMatrix{T,<:HIPData},
                            b::PVector{T,<:HIPData}, α::Number, β::Number) where T
  @check oids_are_equal(c.rows, a.rows)
  @check oids_are_equal(a.cols, b.rows)
  @check hids_are_equal(a.cols, b.rows)
  A, yv, yi, xv, xi, xg = dev_mat(a), dev_vec(c), dev_idx(c.rows), dev_vec(b), dev_idx(b.rows), dev_xchg(b.rows)
  al = Ref{T}(T(α)); be = Ref{T}(T(β))
  check(ccall((:pa_spmv_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}},
               Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ref{T}, Ref{T}),
              length(A), A, yv, yi, xv, xi, xg, al, be))
  mark_device_dirty!(c); mark_device_dirty!(b)   # b's ghost values were exchanged
  c
end

# exchange!(v) / assemble!(v) (Interfaces.jl:2071-2106)
function PartitionedArrays.exchange!(v::PVector{T,<:HIPData}) where T
  vv, vi, xg = dev_vec(v), dev_idx(v.rows), dev_xchg(v.rows)
  check(ccall((:pa_exchange_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Cint, Cint, Cint),
              length(vv), vv, xg, vi, 0, 0, 0))
  mark_device_dirty!(v); v
end
function PartitionedArrays.assemble!(v::PVector{T,<:HIPData}) where T
  vv, vi, xg = dev_vec(v), dev_idx(v.rows), dev_xchg(v.rows)
  check(ccall((:pa_exchange_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Cint, Cint, Cint),
              length(vv), vv, xg, vi, 1, 1, 1))
  mark_device_dirty!(v); v
end

# exchange!(A) / assemble!(A) over nonzeros (Interfaces.jl:2375-2404); the
# matrix exchanger (2300-2372) is built on the host as the reference does and
# handed over with its Int64 nz ids.
function pa_mat_xchg(A::Ptr{Cvoid}, ex::Exchanger, part)
  out = Ref{Ptr{Cvoid}}(C_NULL)
  lr, ls = ex.lids_rcv.parts[part], ex.lids_snd.parts[part]
  pr, ps = Int32.(ex.parts_rcv.parts[part]), Int32.(ex.parts_snd.parts[part])
  check(ccall((:pa_mat_xchg_create, libpa), Cint,
              (Ptr{Cvoid}, Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int64},
               Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int64}, Ref{Ptr{Cvoid}}),
              A, length(pr), pr, lr.ptrs, Int64.(lr.data), length(ps), ps, ls.ptrs, Int64.(ls.data), out))
  out[]
end
function PartitionedArrays.exchange!(a::PSparseMatrix{T,<:HIPData}) where T
  A, mx = dev_mat(a), dev_mat_xchg(a)
  check(ccall((:pa_mat_exchange_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Cint, Cint, Cint), length(A), A, mx, 0, 0, 0))
  a
end
function PartitionedArrays.assemble!(a::PSparseMatrix{T,<:HIPData}) where T
  A, mx = dev_mat(a), dev_mat_xchg(a)
  check(ccall((:pa_mat_exchange_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Cint, Cint, Cint), length(A), A, mx, 1, 1, 1))
  a
end

# dot / norm (Interfaces.jl:1767-1772, 1985-1992)
function LinearAlgebra.dot(a::PVector{T,<:HIPData}, b::PVector{T,<:HIPData}) where T
  r = Ref{T}(zero(T))
  check(ccall((:pa_dot_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ref{T}),
              num_parts(a.values), dev_vec(a), dev_idx(a.rows), dev_vec(b), dev_idx(b.rows), r))
  r[]
end
function LinearAlgebra.norm(a::PVector{T,<:HIPData}, p::Real=2) where T
  p == 2 || return invoke(norm, Tuple{PVector,Real}, a, p)
  r = Ref{Float64}(0.0)
  check(ccall((:pa_norm2_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ref{Float64}),
              num_parts(a.values), dev_vec(a), dev_idx(a.rows), r))
  r[]
end

# PSparseMatrix(I, J, V, rows, cols; ids=:local) (Interfaces.jl:2194-2244):
# sparse(I,J,V,m,n,+) on the device; the CSC pattern comes back for the
# host-side matrix_exchanger (2300-2372).
function pa_mat_coo(ctx::PartCtx, I::Vector{Int64}, J::Vector{Int64}, V::Vector{Tv},
                    m::Integer, n::Integer, rows_h, cols_h; ids::Symbol=:local) where Tv
  out = Ref{Ptr{Cvoid}}(C_NULL)
  nnz = Ref{Int64}(0)
  colptr = Vector{Int64}(undef, n + 1)
  rowval = Vector{Int64}(undef, length(I))
  check(ccall((:pa_mat_from_coo, libpa), Cint,
              (Ptr{Cvoid}, Cint, Cint, Cint, Int64, Int64, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Tv},
               Ptr{Cvoid}, Ptr{Cvoid}, Ref{Int64}, Ptr{Int64}, Ptr{Int64}, Ref{Ptr{Cvoid}}),
              ctx.h, dtype_code(Tv), 8, ids === :global ? 1 : 0, m, n, length(I), I, J, V, rows_h, cols_h,
              nnz, colptr, rowval, out))
  out[], colptr, resize!(rowval, nnz[])
end

# IterativeSolvers.cg! (v0.9) on HIP parts: the whole recurrence on the device
# (scalars included); same iterates as the generic cg! over mul!/dot/norm.
function IterativeSolvers.cg!(x::PVector{T,<:HIPData}, A::PSparseMatrix{T,<:HIPData},
                              b::PVector{T,<:HIPData};
                              abstol::Real=zero(real(T)), reltol::Real=sqrt(eps(real(T))),
                              maxiter::Int=size(A, 2), log::Bool=false, kwargs...) where T
  u, r, c = similar(x), similar(x), similar(x)
  bb = b.rows === x.rows ? b : copyto!(similar(x), b)
  its = Ref{Int64}(0); res = Ref{Float64}(0.0)
  hist = log ? Vector{Float64}(undef, maxiter) : Ptr{Float64}(C_NULL)
  check(ccall((:pa_cg_solve_all, libpa), Cint,
              (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}},
               Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}},
               Float64, Float64, Int64, Cint, Ref{Int64}, Ref{Float64}, Ptr{Float64}),
              num_parts(x.values), dev_mat(A), dev_vec(x), dev_vec(bb), dev_vec(u), dev_vec(r),
              dev_vec(c), dev_idx(x.rows), dev_xchg(x.rows), reltol, abstol, maxiter, 16, its, res, hist))
  mark_host_dirty!(x)
  log ? (x, resize!(hist, its[])) : x
end

# dev_vec / dev_idx / dev_xchg / dev_mat / mark_device_dirty!: the handle
# cache and host/device coherence (INTEGRATION.md §3) — omitted here.

end # module
