// Device-side serving chain (serve/fastpath.py): the kernels of one hop of a request through
// the rank chain, with no host round trip between stages.
//
// The reference forwards every request hop by hop with a blocking gRPC call per stage
// (/root/reference/src/grpc_node.py:120-135, 10 s deadline per hop). Here stage k's stream
// holds, per request: chain_wait (its input slot's flag reached the request's sequence number)
// -> the stage's GEMV layers -> chain_send (wait until the consumer has freed the slot this
// request reuses, copy the rows into the consumer's IPC-mapped slot, write the slot header,
// release the consumer's flag and the producer's ack). Stage k's host enqueues that as soon as
// the request is announced, so every stage's kernels are queued before the data arrives.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dnn {

// Slot header status codes (low 8 bits; bits 8..15: the stage blamed -- the failing stage, the
// producer whose rows never arrived, or the consumer that never freed its slot).
constexpr uint32_t CHAIN_OK = 0, CHAIN_VALUE = 2, CHAIN_INTERNAL = 3, CHAIN_DEADLINE = 4;

struct ChainSend {
  const void* src;           // rows x row_bytes, leading dimension src_ld bytes
  long src_ld;
  void* dst;                 // consumer's slot (IPC-mapped), leading dimension dst_ld bytes
  long dst_ld;
  int rows;                  // rows to copy (0: status only)
  int row_bytes;             // multiple of 16
  uint32_t* dst_hdr;         // consumer's slot header [status, rows]
  const uint32_t* in_hdr;    // this stage's input slot header (nullptr on stage 0)
  uint32_t* err;             // this stage's wait-timeout word (read and cleared here)
  int stage;                 // this stage's index (recorded with a status it raises)
  uint32_t status;           // != 0: raise this status (host-detected failure), copy nothing
  const uint32_t* ack;       // consumer's "slot consumed" flag (written by the consumer)
  uint32_t ack_target;       // wait until ack >= this before overwriting the slot
  uint32_t* next_flag;       // consumer's input flag for this slot
  uint32_t seq;              // this request's sequence number
  uint32_t* prev_ack;        // producer's ack flag (this stage consumed its input slot)
  unsigned long long timeout_ticks;
};

// Receive side of a hop: one lane spins on the input slot's flag (>= seq); then the workgroup
// pulls the slot's rows and header into this stage's own (L2-cached) buffers and releases the
// producer's ack (the slot may be reused). On timeout: *err = 1, nothing is pulled or acked.
struct ChainRecv {
  const uint32_t* flag;      // this stage's input flag of the slot (written by the producer)
  const void* slot;          // the slot's rows (L2-uncached), leading dimension slot_ld bytes
  long slot_ld;
  const uint32_t* slot_hdr;  // the slot's header [status, rows]
  void* dst;                 // this stage's input buffer, leading dimension dst_ld bytes
  long dst_ld;
  uint32_t* dst_hdr;         // local copy of the header (read by this stage's chain_send)
  int rows, row_bytes;
  uint32_t* err;
  uint32_t seq;
  uint32_t* prev_ack;        // producer's ack flag (IPC-mapped)
  unsigned long long timeout_ticks;
};

int chain_recv(const ChainRecv& p, hipStream_t stream);
unsigned long long chain_ticks(double seconds);  // wall_clock64 ticks

// Spin (one lane, s_sleep between system-scope acquire polls) until *flag >= target (wrapping
// compare); *err = 0 when it arrived, 1 when it gave up after timeout_ticks (every wave always
// finishes).
int chain_wait(const uint32_t* flag, uint32_t target, uint32_t* err, double timeout_s,
               hipStream_t stream);
int chain_send(const ChainSend& p, hipStream_t stream);
// *flag = value with system-scope release (one lane, a vector store).
int chain_signal(uint32_t* flag, uint32_t value, hipStream_t stream);

// A stage's LAST serving layer fused with the send of its hop: the GEMV of gemv.hip (one wave
// per output neuron, bias + activation) writes its rows straight into the consumer's
// IPC-mapped slot instead of a local buffer, and the last workgroup to finish (a counter, as
// in p2p_copy_signal_seq) writes the slot header and releases the consumer's flag -- one
// launch and no row copy instead of gemv + chain_send. Status / blame as chain_send: an
// upstream failure or a missed input travels on, a consumer that never freed the slot
// (ack timeout in any workgroup) is blamed, and then no workgroup writes rows.
// With `in_flag` set the receive is folded in too (one kernel per hop): every workgroup
// waits for the input slot's flag (>= seq) and reads the rows straight from the slot (`x`,
// L2-uncached); `in_hdr` is then the slot's header, and the last workgroup also releases the
// producer's ack (`prev_ack`: every workgroup has read the slot). A missed input blames the
// producer, as chain_recv + chain_send do.
struct ChainGemvSend {
  const uint32_t* in_flag;   // nullptr: x is already local (chain_recv ran, or stage 0)
  const uint16_t* x;         // [rows][ldx] bf16 input rows
  long ldx;
  const uint16_t* w;         // [N][ldw] bf16 weights (nn.Linear layout)
  long ldw;
  const float* bias;         // [N] or nullptr
  int act;                   // Act code (forward activation)
  int rows, N, K;            // rows <= GEMV_MAX_ROWS; K % 8 == 0
  int out_f32;               // the slot holds fp32 (else bf16) rows
  void* dst;                 // consumer's slot, leading dimension dst_ld ELEMENTS
  long dst_ld;
  uint32_t* dst_hdr;
  const uint32_t* in_hdr;
  uint32_t* err;
  int stage;
  uint32_t status;
  const uint32_t* ack;
  uint32_t ack_target;
  uint32_t* next_flag;
  uint32_t seq;
  uint32_t* prev_ack;
  uint32_t* counter;         // [2] zero-initialised, left zeroed: arrivals, ack failures
  unsigned long long timeout_ticks;
};
int chain_gemv_send(const ChainGemvSend& p, hipStream_t stream);

// Persistent stage of the serving chain (one-layer stages > 0): ONE launch serves request after
// request with no host work per request. Workgroup 0 polls the input flag of the next slot
// (and the stop word, and an idle timer) and releases the other workgroups through `go`; every
// workgroup stages the slot's rows in LDS, computes its share of the layer (chain_gemv_send's
// math, bitwise), writes straight into the consumer's slot and counts in on the slot's
// counter; the last one writes the header, raises the consumer's flag, acks the producer and
// publishes `done`. The rows of a request come from the slot header its producer wrote. The
// kernel returns when the host sets `*stop` or after `idle_ticks` without a request (the host
// relaunches it with start_seq = *done); either way every wave leaves through the same
// decision of workgroup 0.
struct ChainStage {
  const uint32_t* in_flags;  // [nslot] this stage's input flags (written by the producer)
  const uint32_t* in_hdrs;   // [nslot][2] input slot headers (status, rows)
  const uint16_t* in_slots;  // [nslot][max_rows][ldx] bf16 rows (L2-uncached)
  long ldx;                  // elements (= K padded)
  uint32_t* prev_ack;        // producer's ack word (IPC-mapped)
  const uint16_t* w;         // [N][ldw]
  long ldw;
  const float* bias;
  int act;                   // Act code; ACT_SOFTMAX: row softmax (one workgroup, N <= 1024)
  int N, K;
  int out_f32;
  char* dst;                 // consumer's slot 0 rows; slot s at dst + s * dst_slot_bytes
  long dst_slot_bytes;
  long dst_ld;               // elements
  uint32_t* dst_hdr;         // consumer's slot 0 header; slot s at dst_hdr + s * hdr_stride
  long hdr_stride;           // words
  uint32_t* next_flags;      // [nslot] the consumer's flags for the slots
  const uint32_t* ack;       // this stage's ack word (the consumer writes it)
  const uint32_t* stop;      // != 0 -> return (coherent host memory, set by the host)
  uint32_t* done;            // the last request finished (coherent host memory: progress)
  uint32_t* sync;            // [2 nslot + 4] zeroed: per-slot arrival counters, per-slot ack
                             // failures, go, exit (+ exit reason, its value)
  uint32_t start_seq;        // serve start_seq + 1, start_seq + 2, ...
  uint32_t epoch;            // this launch's id (exit word value)
  int stage, nslot, max_rows;
  unsigned long long idle_ticks, timeout_ticks;
};
// Returns the workgroups launched (>= 1; capped so that `share` persistent stages on this GPU
// are all resident at once) or < 0 on a parameter / launch error.
int chain_stage_run(const ChainStage& p, int workgroups, int share, hipStream_t stream);
int chain_stage_workgroups(int N, int act);  // the grid chain_stage_run is given by default

// Training step plans (runtime/step_plan.cpp COPYSIG): a peer copy followed by its flag in ONE
// launch. Every workgroup copies its share, fences, and bumps `counter`; the last one to
// arrive resets the counter and stores *flag = *seq + delta (system-scope release), so the
// flag is raised only after every workgroup's rows are visible. `counter` starts at 0 and is
// left at 0.
int p2p_copy_signal_seq(void* dst, const void* src, size_t bytes, uint32_t* flag,
                        const uint32_t* seq, int delta, uint32_t* counter, hipStream_t stream);

}  // namespace dnn
