// Device-side serving chain kernels (chain.hpp; host side serve/fastpath.py). Every wait is a
// single lane polling a flag with system-scope acquire loads and s_sleep between polls, with a
// wall-clock timeout, so every wave of every launch finishes. Flags and slot headers are
// written with vector stores (the address is lane-indexed), never through the scalar cache.
#include <algorithm>

#include "chain.hpp"
#include "common.hpp"
#include "gemv.hpp"

namespace dnn {

namespace {

bool misaligned4(const void* p) { return reinterpret_cast<uintptr_t>(p) & 3; }
bool misaligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) & 15; }

__device__ __forceinline__ bool reached(const uint32_t* flag, uint32_t target) {
  return (int)(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - target) >=
         0;
}

// lane 0 of the calling wave: poll until reached or timed out. `relaxed`: a long sleep
// between polls (~1000 clocks instead of ~64), for the many workgroups of a one-launch hop
// that all wait on one flag -- their uncached polls otherwise flood the memory system the
// flag's own write has to get through (profiles/r4_chain: 4 waiting stages, 144 vs 18 us)
template <bool relaxed = false>
__device__ __forceinline__ bool spin(const uint32_t* flag, uint32_t target,
                                     unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (!reached(flag, target)) {
    if constexpr (relaxed) __builtin_amdgcn_s_sleep(16);
    else __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > ticks) return false;
  }
  return true;
}

// rows x row_bytes from src (ld sld bytes) to dst (ld dld bytes), 16-byte vectors
__device__ __forceinline__ void copy_rows(const char* src, long sld, char* dst, long dld,
                                          int rows, int row_bytes) {
  const int cpr = row_bytes >> 4;
  const int n = rows * cpr;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int r = i / cpr, c = i - r * cpr;
    *(uint4*)(dst + r * dld + 16 * c) = *(const uint4*)(src + r * sld + 16 * c);
  }
}

}  // namespace

__global__ void chain_wait_kernel(const uint32_t* flag, uint32_t target, uint32_t* err,
                                  unsigned long long ticks) {
  const unsigned l = threadIdx.x;
  if (l != 0) return;
  const bool ok = spin(flag + l, target, ticks);  // err: this wait's outcome (0 = arrived)
  __hip_atomic_store(err + l, ok ? 0u : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void chain_recv_kernel(ChainRecv p) {
  __shared__ uint32_t s_ok;
  const unsigned t = threadIdx.x;
  if (t == 0) {
    const bool ok = spin(p.flag + t, p.seq, p.timeout_ticks);
    if (!ok) __hip_atomic_store(p.err + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s_ok = ok ? 1u : 0u;
  }
  __syncthreads();
  if (!s_ok) return;  // uniform
  copy_rows((const char*)p.slot, p.slot_ld, (char*)p.dst, p.dst_ld, p.rows, p.row_bytes);
  if (t < 2)
    p.dst_hdr[t] = __hip_atomic_load(p.slot_hdr + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // every read of the slot is done before the producer may overwrite it
  __syncthreads();
  if (t == 0 && p.prev_ack) {
    __threadfence_system();
    __hip_atomic_store(p.prev_ack + t, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(256) void chain_send_kernel(ChainSend p) {
  __shared__ uint32_t s_st;
  const unsigned t = threadIdx.x;
  if (t == 0) {
    bool ok = true;
    if (p.ack) ok = spin(p.ack + t, p.ack_target, p.timeout_ticks);
    uint32_t st = p.status;
    if (!st) {
      const uint32_t in = p.in_hdr ? p.in_hdr[t] : 0u;
      if (in & 0xffu)  // an upstream failure travels on unchanged (it names its stage)
        st = in;
      else if (__hip_atomic_load(p.err + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
        st = CHAIN_DEADLINE | ((uint32_t)(p.stage - 1) << 8);  // the producer never delivered
      else if (!ok)
        st = CHAIN_DEADLINE | ((uint32_t)(p.stage + 1) << 8);  // the consumer never drained
    }
    __hip_atomic_store(p.err + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s_st = st | (ok ? 0u : 0x80000000u);
  }
  __syncthreads();
  const uint32_t st = s_st & 0x7fffffffu;
  const bool slot_free = (s_st & 0x80000000u) == 0u;
  if (st == 0u && slot_free)
    copy_rows((const char*)p.src, p.src_ld, (char*)p.dst, p.dst_ld, p.rows, p.row_bytes);
  if (t < 2)
    __hip_atomic_store(p.dst_hdr + t, t == 0 ? st : (uint32_t)p.rows, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();  // this thread's rows and header are visible before the flag
  __syncthreads();
  if (t == 0)
    __hip_atomic_store(p.next_flag + t, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t == 1 && p.prev_ack)
    __hip_atomic_store(p.prev_ack + (t - 1), p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The status a hop sends on (chain_send's rule): an upstream failure travels on unchanged,
// a missed input blames the producer, an ack timeout the consumer.
__device__ __forceinline__ uint32_t hop_status(uint32_t status, const uint32_t* in_hdr,
                                               const uint32_t* err, int stage, bool ack_ok,
                                               unsigned t, bool in_ok = true) {
  if (status) return status;
  if (!in_ok) return CHAIN_DEADLINE | ((uint32_t)(stage - 1) << 8);  // input never came
  const uint32_t in = in_hdr ? __hip_atomic_load(in_hdr + t, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
  if (in & 0xffu) return in;
  if (__hip_atomic_load(err + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
    return CHAIN_DEADLINE | ((uint32_t)(stage - 1) << 8);
  if (!ack_ok) return CHAIN_DEADLINE | ((uint32_t)(stage + 1) << 8);
  return 0u;
}

constexpr int CG_WAVES = 4;  // output neurons (waves) per 256-thread workgroup, as gemv.hip

template <int M, bool OUT_F32>
__global__ __launch_bounds__(256) void chain_gemv_send_kernel(ChainGemvSend p) {
  __shared__ uint32_t s_go;
  const unsigned t = threadIdx.x;
  const int lane = t & 63;
  if (t == 0) {
    // the input (folded receive) first, then the consumer's slot; both bounded
    const bool in_ok = !p.in_flag ? true
                       : blockIdx.x == 0 ? spin(p.in_flag + t, p.seq, p.timeout_ticks)
                                         : spin<true>(p.in_flag + t, p.seq, p.timeout_ticks);
    // (the grid can be N / 4 workgroups: all but one poll the consumer's ack relaxed, as the
    // folded receive's input flag, so a wide layer does not flood the memory system)
    const bool ok = !p.ack ? true
                    : blockIdx.x == 0 ? spin(p.ack + t, p.ack_target, p.timeout_ticks)
                                      : spin<true>(p.ack + t, p.ack_target, p.timeout_ticks);
    if (!ok || !in_ok)  // remembered for the last workgroup: bit 0 ack, bit 1 input
      __hip_atomic_fetch_or(p.counter + 1 + t, (ok ? 0u : 1u) | (in_ok ? 0u : 2u),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_go = hop_status(p.status, p.in_hdr, p.err, p.stage, ok, t, in_ok) == 0u ? 1u : 0u;
  }
  __syncthreads();
  // a wave per output neuron; with fewer workgroups than N / 4 (the folded receive: every
  // workgroup spins, so the grid is capped) a wave takes every (grid * 4)-th neuron
  for (int n = blockIdx.x * CG_WAVES + (int)(t >> 6); s_go && n < p.N;
       n += gridDim.x * CG_WAVES) {  // (no early return: every thread reaches the barrier)
    const uint16_t* wr = p.w + (long)n * p.ldw;
    float acc[M];
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m] = 0.f;
    constexpr int U = 4;
    for (int k0 = 0; k0 < p.K; k0 += 512 * U) {
      bf16x8_t wv[U], xv[U][M];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u * 512 + lane * 8;
        if (k < p.K) {
          wv[u] = *(const bf16x8_t*)(wr + k);
#pragma unroll
          for (int m = 0; m < M; ++m)
            xv[u][m] = m < p.rows ? *(const bf16x8_t*)(p.x + m * p.ldx + k) : bf16x8_t{};
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u * 512 + lane * 8;
        if (k < p.K) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float we = bf2f((u16)wv[u][e]);
#pragma unroll
            for (int m = 0; m < M; ++m) acc[m] += we * bf2f((u16)xv[u][m][e]);
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m] = wave_sum(acc[m]);
    if (lane < p.rows) {
      float v = 0.f;
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (m == lane) v = acc[m];
      v = act_fwd(v + (p.bias ? p.bias[n] : 0.f), p.act);
      if constexpr (OUT_F32)
        ((float*)p.dst)[(long)lane * p.dst_ld + n] = v;
      else
        ((u16*)p.dst)[(long)lane * p.dst_ld + n] = f2bf(v);
    }
  }
  __threadfence_system();  // this thread's rows are visible before the workgroup counts in
  __syncthreads();
  if (t == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(p.counter + t, 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {  // the last workgroup: every row has landed
      const uint32_t fail = __hip_atomic_load(p.counter + 1 + t, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t st = hop_status(p.status, p.in_hdr, p.err, p.stage, (fail & 1u) == 0u, t,
                                     (fail & 2u) == 0u);
      __hip_atomic_store(p.counter + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.counter + 1 + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.err + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(p.dst_hdr + t, st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(p.dst_hdr + 1 + t, (uint32_t)p.rows, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
      __hip_atomic_store(p.next_flag + t, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (p.prev_ack)
        __hip_atomic_store(p.prev_ack + t, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---- persistent stage (ChainStage, chain.hpp) ---------------------------------------------
// sync words: [0, nslot) per-slot arrival counters, [nslot, 2 nslot) per-slot ack failures
// (written by workgroup 0 before it releases the slot), then go, exit.

// One request's layer for `rows` <= M rows staged in LDS (xs, row stride K). A wave takes NB
// neurons at once (their weight loads in flight together, the x vectors read once for all);
// per neuron the loop and reduction order are chain_gemv_send's, so the outputs are bitwise
// the same. `logits` != nullptr (softmax, one workgroup): the pre-activation rows go there.
template <int M, int NB>
__device__ __forceinline__ void cs_layer(const ChainStage& p, const u16* xs, int rows, char* dst,
                                         float* logits) {
  const unsigned t = threadIdx.x;
  const int lane = t & 63;
  constexpr int U = 2;  // (the loop order per lane is U-independent: bitwise as U = 4)
  for (int n0 = (blockIdx.x * CG_WAVES + (int)(t >> 6)) * NB; n0 < p.N;
       n0 += gridDim.x * CG_WAVES * NB) {
    float acc[NB][M];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int m = 0; m < M; ++m) acc[j][m] = 0.f;
    for (int k0 = 0; k0 < p.K; k0 += 512 * U) {
      bf16x8_t wv[NB][U], xv[U][M];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u * 512 + lane * 8;
        if (k < p.K) {
#pragma unroll
          for (int j = 0; j < NB; ++j)
            wv[j][u] = n0 + j < p.N ? *(const bf16x8_t*)(p.w + (long)(n0 + j) * p.ldw + k)
                                    : bf16x8_t{};
#pragma unroll
          for (int m = 0; m < M; ++m)
            xv[u][m] = m < rows ? *(const bf16x8_t*)(xs + m * p.K + k) : bf16x8_t{};
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u * 512 + lane * 8;
        if (k < p.K) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
#pragma unroll
            for (int j = 0; j < NB; ++j) {
              const float we = bf2f((u16)wv[j][u][e]);
#pragma unroll
              for (int m = 0; m < M; ++m) acc[j][m] += we * bf2f((u16)xv[u][m][e]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
#pragma unroll
      for (int m = 0; m < M; ++m) acc[j][m] = wave_sum(acc[j][m]);
      const int n = n0 + j;
      if (n < p.N && lane < rows) {
        float v = 0.f;
#pragma unroll
        for (int m = 0; m < M; ++m)
          if (m == lane) v = acc[j][m];
        v += p.bias ? p.bias[n] : 0.f;
        if (logits) {
          logits[lane * p.N + n] = v;
        } else {
          v = act_fwd(v, p.act);
          if (p.out_f32)
            ((float*)dst)[(long)lane * p.dst_ld + n] = v;
          else
            ((u16*)dst)[(long)lane * p.dst_ld + n] = f2bf(v);
        }
      }
    }
  }
}

constexpr int CS_NB = 4;  // neurons per wave in flight (chain_stage_kernel)

__global__ __launch_bounds__(256) void chain_stage_kernel(ChainStage p) {
  extern __shared__ __attribute__((aligned(16))) char cs_lds[];
  __shared__ uint32_t s_cmd[4];  // run, input status, rows, ack failure
  u16* xs = (u16*)cs_lds;
  float* logits = p.act == ACT_SOFTMAX ? (float*)(cs_lds + (long)p.max_rows * p.K * 2) : nullptr;
  const unsigned t = threadIdx.x;
  uint32_t* cnt = p.sync;
  uint32_t* fail = p.sync + p.nslot;
  uint32_t* go = p.sync + 2 * p.nslot;  // workgroup 0: the last request it let through
  uint32_t* ex = go + 1;                // == epoch: this launch ends before request *go + 1
                                        // (ex[1]: why -- 1 stop, 2 idle; ex[2]: the stop
                                        // word read / the idle ticks)
  uint32_t stop_seen = 0;  // workgroup 0: the stop word read after the last request's go
  for (uint32_t seq = p.start_seq + 1;; ++seq) {
    const int slot = (int)(seq % (uint32_t)p.nslot);
    if (t == 0) {
      uint32_t run = 1;
      if (blockIdx.x == 0 && stop_seen) {  // asked to stop while the last request ran
        run = 0;
        __hip_atomic_store(ex + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ex + 2, stop_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ex, p.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else if (blockIdx.x == 0) {
        // the consumer drained the slot this request will reuse -- checked BEFORE the input
        // arrives (it nearly always has: the wait is off the request's path). Bounded: a stuck
        // consumer is reported downstream as DEADLINE naming it, no rows are written.
        // The stop word lives in host memory (a read crosses the host link): looked at every
        // ~20 us of waiting, not every poll of a (local) flag -- in this ack wait too, so a
        // stage whose consumer is stuck still returns promptly when asked.
        bool ack_ok = true;
        unsigned long long t_stop = wall_clock64();
        {
          const unsigned long long ta = t_stop;
          while ((int)(__hip_atomic_load(p.ack, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                       (seq - (uint32_t)p.nslot)) < 0) {
            const unsigned long long now = wall_clock64();
            if (now - t_stop > 2000) {
              t_stop = now;
              const uint32_t sv = __hip_atomic_load(p.stop, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_SYSTEM);
              if (sv) {  // the exit reason is recorded as on the input-wait path
                run = 0;
                __hip_atomic_store(ex + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(ex + 2, sv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
              }
            }
            if (now - ta > p.timeout_ticks) {
              ack_ok = false;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        const unsigned long long t0 = wall_clock64();
        for (; run;) {
          if ((int)(__hip_atomic_load(p.in_flags + slot, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM) - seq) >= 0)
            break;
          const unsigned long long now = wall_clock64();
          if (now - t_stop > 2000) {
            t_stop = now;
            const uint32_t sv = __hip_atomic_load(p.stop, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM);
            if (sv) {
              run = 0;
              __hip_atomic_store(ex + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(ex + 2, sv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
          }
          if (now - t0 > p.idle_ticks) {
            run = 0;
            __hip_atomic_store(ex + 1, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ex + 2, (uint32_t)(now - t0), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (run) {
          __hip_atomic_store(fail + slot, ack_ok ? 0u : 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(go, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          // one look at the stop word per request, off the request's path (the other
          // workgroups are already computing): back-to-back requests never wait the ~20 us
          // the polls above need before they read it, so a paused() chain would otherwise
          // run until its hop timeout
          stop_seen = __hip_atomic_load(p.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
          __hip_atomic_store(ex, p.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        // the other workgroups follow workgroup 0's decision (it alone polls the input flag
        // and owns the idle / stop exit, so every workgroup leaves at the same request)
        for (;;) {
          if ((int)(__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - seq) >= 0)
            break;
          if (__hip_atomic_load(ex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p.epoch) {
            run = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (run) {
        // no acquire fence: it would invalidate the L2 that keeps this stage's weights resident
        // between requests. The header and rows are read with system-scope loads instead
        // (they bypass every cache level), issued after the flag / go was seen.
        s_cmd[1] = __hip_atomic_load(p.in_hdrs + 2 * slot, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
        s_cmd[2] = __hip_atomic_load(p.in_hdrs + 2 * slot + 1, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
        s_cmd[3] = __hip_atomic_load(fail + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      s_cmd[0] = run;
    }
    __syncthreads();
    if (!s_cmd[0]) break;  // uniform: the launch ends here
    const uint32_t in_st = s_cmd[1];
    const int rows = (int)s_cmd[2];
    const bool rows_ok = rows >= 1 && rows <= p.max_rows;
    const uint32_t ack_fail = s_cmd[3];
    const bool compute = (in_st & 0xffu) == 0u && ack_fail == 0u && rows_ok;
    char* dst = p.dst + slot * p.dst_slot_bytes;
    if (compute) {
      const u16* src = p.in_slots + (long)slot * p.max_rows * p.ldx;
      const int cpr = p.K >> 2;  // 8-byte words per row
      for (int i = t; i < rows * cpr; i += blockDim.x) {
        const int r = i / cpr, c = i - r * cpr;
        *(uint64_t*)(xs + r * p.K + 4 * c) = __hip_atomic_load(
            (const uint64_t*)(src + r * p.ldx + 4 * c), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __syncthreads();
      switch (rows) {
        case 1: cs_layer<1, CS_NB>(p, xs, rows, dst, logits); break;
        case 2: cs_layer<2, CS_NB>(p, xs, rows, dst, logits); break;
        case 3:
        case 4: cs_layer<4, CS_NB>(p, xs, rows, dst, logits); break;
        default: cs_layer<8, CS_NB>(p, xs, rows, dst, logits); break;
      }
      if (logits) {  // row softmax (one workgroup): a wave per row
        __syncthreads();
        const int lane = t & 63;
        for (int m = (int)(t >> 6); m < rows; m += CG_WAVES) {
          float mx = -INFINITY;
          for (int n = lane; n < p.N; n += 64) mx = fmaxf(mx, logits[m * p.N + n]);
          mx = wave_max(mx);
          float s = 0.f;
          for (int n = lane; n < p.N; n += 64) s += __expf(logits[m * p.N + n] - mx);
          s = wave_sum(s);
          const float inv = 1.f / s;
          for (int n = lane; n < p.N; n += 64) {
            const float v = __expf(logits[m * p.N + n] - mx) * inv;
            if (p.out_f32)
              ((float*)dst)[(long)m * p.dst_ld + n] = v;
            else
              ((u16*)dst)[(long)m * p.dst_ld + n] = f2bf(v);
          }
        }
      }
    }
    // this thread's rows are visible before the workgroup counts in: a release-only fence
    // (a full __threadfence_system would also invalidate the L2 holding the weights)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (t == 0) {
      // acq_rel at agent scope: every workgroup's release (fence above) synchronizes with
      // the last arriver's acquire, so the rows it publishes below are ordered by the memory
      // model, not only by each writer's own fence. An agent-scope acquire invalidates the
      // per-CU caches only, not the L2 that keeps this stage's weights resident
      const uint32_t prev = __hip_atomic_fetch_add(cnt + slot, 1u, __ATOMIC_ACQ_REL,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      if (prev == gridDim.x - 1) {  // the last workgroup: every row of the request landed
        uint32_t st = 0u;
        if (in_st & 0xffu) st = in_st;  // an upstream failure travels on unchanged
        else if (ack_fail) st = CHAIN_DEADLINE | ((uint32_t)(p.stage + 1) << 8);
        else if (!rows_ok) st = CHAIN_INTERNAL | ((uint32_t)p.stage << 8);
        __hip_atomic_store(cnt + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t* hdr = p.dst_hdr + slot * p.hdr_stride;
        __hip_atomic_store(hdr, st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(hdr + 1, (uint32_t)(rows_ok ? rows : 0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(p.next_flags + slot, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(p.prev_ack, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(p.done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

__global__ void chain_signal_kernel(uint32_t* flag, uint32_t value) {
  const unsigned l = threadIdx.x;
  if (l == 0) {
    __threadfence_system();
    __hip_atomic_store(flag + l, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(256) void p2p_copy_signal_seq_kernel(
    const uint4* __restrict__ src, uint4* __restrict__ dst, long n16,
    const unsigned char* __restrict__ src_t, unsigned char* __restrict__ dst_t, int tail,
    uint32_t* flag, const uint32_t* seq, int delta, uint32_t* counter) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256)
    dst[i] = src[i];
  if (blockIdx.x == 0 && (int)threadIdx.x < tail) dst_t[threadIdx.x] = src_t[threadIdx.x];
  __threadfence_system();  // this thread's part is visible before the workgroup counts in
  __syncthreads();
  const unsigned t = threadIdx.x;
  if (t == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(counter + t, 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {  // the last workgroup: every part has landed
      __hip_atomic_store(counter + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t v = __hip_atomic_load(seq + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(flag + t, v + (uint32_t)delta, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

int p2p_copy_signal_seq(void* dst, const void* src, size_t bytes, uint32_t* flag,
                        const uint32_t* seq, int delta, uint32_t* counter, hipStream_t stream) {
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) return -1;
  if (!flag || !seq || !counter || misaligned4(flag) || misaligned4(counter)) return -1;
  const long n16 = (long)(bytes / 16);
  const int tail = (int)(bytes % 16);
  const int grid = (int)std::min<long>(std::max<long>(1, (n16 + 255) / 256), 2048);
  hipLaunchKernelGGL(p2p_copy_signal_seq_kernel, dim3(grid), dim3(256), 0, stream,
                     reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), n16,
                     reinterpret_cast<const unsigned char*>(src) + n16 * 16,
                     reinterpret_cast<unsigned char*>(dst) + n16 * 16, tail, flag, seq, delta,
                     counter);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

unsigned long long chain_ticks(double seconds) {
  static int rate_khz = [] {  // wall_clock64 ticks per ms (100 MHz on gfx9)
    int r = 0, dev = 0;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&r, hipDeviceAttributeWallClockRate, dev);
    return r > 0 ? r : 100000;
  }();
  return (unsigned long long)(std::max(0.0, seconds) * 1e3 * (double)rate_khz);
}


int chain_wait(const uint32_t* flag, uint32_t target, uint32_t* err, double timeout_s,
               hipStream_t stream) {
  if (!flag || !err || misaligned4(flag) || misaligned4(err)) return -1;
  hipLaunchKernelGGL(chain_wait_kernel, dim3(1), dim3(64), 0, stream, flag, target, err,
                     chain_ticks(timeout_s));
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int chain_recv(const ChainRecv& p, hipStream_t stream) {
  if (!p.flag || !p.err || !p.dst_hdr || !p.slot_hdr || misaligned4(p.flag)) return -1;
  if (p.rows < 0 || p.row_bytes % 16 || p.slot_ld % 16 || p.dst_ld % 16 ||
      misaligned16(p.slot) || misaligned16(p.dst))
    return -2;
  hipLaunchKernelGGL(chain_recv_kernel, dim3(1), dim3(256), 0, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int chain_send(const ChainSend& p, hipStream_t stream) {
  if (!p.next_flag || !p.dst_hdr || !p.err || misaligned4(p.next_flag)) return -1;
  if (p.rows < 0 || p.row_bytes % 16 || p.src_ld % 16 || p.dst_ld % 16 ||
      misaligned16(p.src) || misaligned16(p.dst))
    return -2;
  hipLaunchKernelGGL(chain_send_kernel, dim3(1), dim3(256), 0, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int chain_gemv_send(const ChainGemvSend& p, hipStream_t stream) {
  if (!p.next_flag || !p.dst_hdr || !p.err || !p.counter || !p.dst || !p.x || !p.w ||
      misaligned4(p.next_flag) || misaligned4(p.counter))
    return -1;
  if (p.rows < 1 || p.rows > GEMV_MAX_ROWS || p.N < 1 || p.K < 8 || p.K % 8 || p.ldx < p.K ||
      p.ldw < p.K || p.ldx % 8 || p.ldw % 8 || p.dst_ld < p.N || misaligned16(p.x) ||
      misaligned16(p.w))
    return -2;
  // the folded receive makes every workgroup wait on the input flag: at most CG_RECV_WG of
  // them, so a node's worth of waiting stages (a one-GPU rehearsal puts 8 on one GPU) stays
  // far below what the GPU holds at once
  constexpr int CG_RECV_WG = 64;
  const int wg = (p.N + CG_WAVES - 1) / CG_WAVES;
  const dim3 grid(p.in_flag ? std::min(wg, CG_RECV_WG) : wg), block(256);
#define DNN_CG(MM)                                                                           \
  if (p.out_f32)                                                                             \
    hipLaunchKernelGGL((chain_gemv_send_kernel<MM, true>), grid, block, 0, stream, p);       \
  else                                                                                       \
    hipLaunchKernelGGL((chain_gemv_send_kernel<MM, false>), grid, block, 0, stream, p);
  switch (p.rows) {
    case 1: DNN_CG(1) break;
    case 2: DNN_CG(2) break;
    case 3:
    case 4: DNN_CG(4) break;
    default: DNN_CG(8) break;
  }
#undef DNN_CG
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int chain_stage_workgroups(int N, int act) {
  if (act == ACT_SOFTMAX) return 1;  // the row pass needs every logit in one workgroup
  // a neuron group (CS_NB neurons) per wave, at most 64 workgroups: a one-GPU rehearsal keeps
  // 7 persistent stages resident at once (448 workgroups, far below the GPU's ~2048)
  return std::max(1, std::min(64, (N + CG_WAVES * CS_NB - 1) / (CG_WAVES * CS_NB)));
}

int chain_stage_run(const ChainStage& p, int workgroups, int share, hipStream_t stream) {
  if (!p.in_flags || !p.in_hdrs || !p.in_slots || !p.prev_ack || !p.w || !p.dst || !p.dst_hdr ||
      !p.next_flags || !p.ack || !p.stop || !p.done || !p.sync || misaligned4(p.in_flags) ||
      misaligned4(p.sync) || misaligned4(p.next_flags) || misaligned4(p.dst_hdr))
    return -1;
  if (p.N < 1 || p.K < 8 || p.K % 8 || p.ldx < p.K || p.ldx % 8 || p.ldw < p.K || p.ldw % 8 ||
      p.dst_ld < p.N || p.nslot < 2 || p.max_rows < 1 || p.max_rows > GEMV_MAX_ROWS ||
      misaligned16(p.in_slots) || misaligned16(p.w) || p.epoch == 0)
    return -2;
  const long lds = (long)p.max_rows * p.K * 2 +
                   (p.act == ACT_SOFTMAX ? (long)p.max_rows * p.N * 4 : 0);
  if (lds > 64 * 1024) return -3;  // rows staged in LDS: K (and a softmax's N) bounded
  if (workgroups < 1 || (p.act == ACT_SOFTMAX && workgroups != 1)) return -4;
  // every workgroup of every persistent stage on this GPU must be resident at once (a request
  // completes only when all of a stage's workgroups count in, and resident ones never yield):
  // `share` stages split what the GPU holds, with a quarter kept for everything else
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_stage_kernel, 256,
                                                   (size_t)lds) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -9;
  const int cap = std::max(1, per_cu * cus * 3 / 4 / std::max(1, share));
  workgroups = std::min(workgroups, cap);
  hipLaunchKernelGGL(chain_stage_kernel, dim3(workgroups), dim3(256), (size_t)lds, stream, p);
  return hipGetLastError() == hipSuccess ? workgroups : -9;
}

int chain_signal(uint32_t* flag, uint32_t value, hipStream_t stream) {
  if (!flag || misaligned4(flag)) return -1;
  hipLaunchKernelGGL(chain_signal_kernel, dim3(1), dim3(64), 0, stream, flag, value);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

}  // namespace dnn
