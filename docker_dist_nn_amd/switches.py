"""Every behaviour switch of the framework, in one registry.

The reference steers itself with module constants, argparse flags and a per-stage env contract
(/root/reference/src/run_grpc_fcnn.py:17-27, /root/reference/src/grpc_node.py:18-57). Ours adds
engine / kernel switches for A/B measurements and fault injection; they are all declared here
with their default and meaning, read through :func:`get` (the environment is consulted on every
call, so tests can monkeypatch), and reported by :func:`active` -- the benchmark JSON echoes the
switches in effect for its run. Nothing else in the package reads ``DNN_*`` variables.
"""
from __future__ import annotations

import os

SWITCHES: dict[str, tuple[str, str]] = {
    # kernels / tuning
    "DNN_TUNED": ("1", "0 = ignore the tuned GEMM table (ops/tuned_gfx950.json)"),
    "DNN_TUNED_TABLE": ("", "path of another tuned table (A/B of two tunings)"),
    "DNN_BLAS": ("", "hipBLASLt comparison path: '' never (own kernels), 1 = every product "
                     "it supports, or per kind 'fwd=1,dgrad=0,wgrad=1' (bench only)"),
    "DNN_GEMM_EPI_GENERIC": ("0", "1 = the register-direct GEMM epilogue reads the activation per "
                                  "element (the pre-round-4 form; A/B only)"),
    "DNN_GEMM_STAGES": ("", "LDS pipeline depth per GEMM kind ('3' or 'fwd=3,dgrad=2'); 8 = "
                            "ping-pong 256x256 form"),
    "DNN_GEMM_PERSIST": ("", "persistent-workgroup GEMM form per kind ('1', 'fwd=1,wgrad=0')"),
    "DNN_WGRAD_GROUP_MAX_WG": ("256", "grouped wgrad launch: size bound in workgroups"),
    # engine
    "DNN_DGRAD_WT": ("1", "dgrad reads the transposed weight shadow W^T (0 = transpose per tile)"),
    "DNN_WGRAD_KK": ("auto", "K-major weight gradients from transposed dZ / X copies written by "
                             "the producing GEMMs: auto (layers >= 16M weights) | 1 | 0"),
    "DNN_TAIL": ("1", "fused classifier tail kernel (mlp_tail.hip)"),
    "DNN_FUSED_XENT": ("1", "softmax cross-entropy fused into the logits GEMM epilogue"),
    "DNN_RELU_MASK": ("auto", "1-bit ReLU masks instead of the activation in dgrad epilogues: "
                                 "1 = row-block-major bytes, 2 = fragment order (ops.FragMask, "
                                 "register-direct tiles only), 0 = off, auto = 2 for hidden "
                                 "layers >= 1024 wide"),
    "DNN_WGRAD_ALGO": ("splitk", "weight-gradient algorithm: splitk | streamk"),
    "DNN_WGRAD_GROUP": ("1", "one grouped launch for small split-K weight gradients"),
    "DNN_FUSE_FIN_SGD": ("1", "gradient reduction and optimizer step in one launch (FINO)"),
    "DNN_WGRAD_FUSED_UPDATE": ("1", "one-split weight gradients apply SGD (and write W^T) in "
                                    "their GEMM epilogue; no data parallelism"),
    "DNN_NATIVE_EXEC": ("1", "record each stage's launches once and replay them from C++"),
    "DNN_NATIVE_PLAN": ("1", "single-process pipeline step as one native call"),
    "DNN_LOOPBACK_STREAMS": ("1", "single-process pipeline: one stream per stage, event edges "
                                  "per micro-batch hop (0 = the schedule on one stream)"),
    "DNN_NATIVE_DIST": ("1", "multi-rank step as one StepPlan call (parallel/native_step.py)"),
    "DNN_WGRAD_STREAMS": ("1", "concurrent wgrad streams in native single-process plans"),
    "DNN_BENCH_STEP_EVENTS": ("0", "bench.py: 1 = a HIP event around every timed step; the JSON "
                                   "gets the per-step GPU times (diagnosis)"),
    "DNN_BW_OVERLAP": ("1", "wgrad_i on a side stream concurrent with dgrad_i (1 stage, one "
                            "micro-batch): mlp8 3.43 -> 3.31 ms; 5 = small wgrads on the side, "
                            "W1 then W0 on the main stream (fixes their order); 0 = off. The "
                            "rejected modes 2/3/4/6 were removed in round 6 (profiles/r6_prune)"),
    "DNN_BW_OVERLAP_MIN_ROWS": ("16384", "overlap plans only for steps of at least this many "
                                         "rows (below, the single-stream plan: no event "
                                         "packets, the host cost that bounds small steps; "
                                         "headline model 1024 rows 0.093 -> 0.054 ms, 8192 "
                                         "even, 16384 0.155 vs 0.166 for the overlap)"),
    "DNN_SPLIT_FINO": ("auto", "overlap plans: reduce + update layers 1..L-1 on the side "
                       "stream during W0, only layer 0's after it (SGD); auto = when no layer "
                       "updates in its wgrad epilogue (mlp8 2.918 -> 2.889 ms, headline "
                       "0.350 -> 0.346, wide excluded: 6.04 -> 6.21)"),
    "DNN_FIN_WT": ("1", "the fused reduce + SGD/Adam launch (FINO) also writes the W^T "
                        "shadows of the layers it updates (no transpose launch per step)"),
    "DNN_FAULT_NATIVE_STEP": ("", "fault injection (tests): comma-separated ranks whose "
                                   "native multi-rank step construction raises; all ranks "
                                   "then fall back to the Python executor together"),
    "DNN_H0_DOUBLE": ("1", "single-stage native steps: the layer-0 activation alternates between "
                           "two buffers from step to step (a relocatable Program region), so "
                           "with DNN_XSTEP the next step's layer-0 forward does not wait for "
                           "this step's side-stream weight gradient that reads it"),
    "DNN_XSTEP": ("1", "single-stage overlap plans: the next step's layer-0 forward starts "
                       "beside this step's side-stream tail (reduce + update of layers "
                       "1..L-1); the join moves in front of the layer-1 forward (1 = on)"),
    "DNN_EVENT_FENCE": ("device", "fork / join events of single-process step plans: device = "
                                  "no system-scope fence at the record (both streams on one "
                                  "GPU), system = HIP's default (cache write-back per record)"),
    "DNN_DP_DEFER": ("1", "deferred data-parallel update (Python executor path)"),
    "DNN_RCCL_PLAN": ("auto", "native RCCL step form: streams (one stream per hop channel) | "
                      "slotted (one RCCL stream, per-slot groups: safe with one resident RCCL "
                      "kernel) | auto (streams when GPU_MAX_HW_QUEUES >= 6)"),
    "DNN_IPC_PLAN": ("streams", "native IPC step form: streams (a stream per direction and relay "
                                "duty) | slotted (ONE stream in global logical-clock order: "
                                "no co-scheduling assumption, a captured graph is one chain)"),
    "DNN_FIRST_STEP_TIMEOUT": ("30", "bench.py: seconds the first multi-rank step may take "
                               "before the plan trace is printed and the run exits"),
    "DNN_LADDER": ("1", "bench.py with WORLD_SIZE > 1: a supervisor per rank runs each attempt "
                        "in fresh child processes and climbs the fallback ladder (ladder.py) "
                        "on a hang or crash; 0 = measure in this process"),
    "DNN_LADDER_STALL": ("60", "ladder: seconds a child may go without a heartbeat before "
                                "it is killed and the next rung runs"),
    "DNN_LADDER_BUDGET": ("360", "ladder: seconds of attempts after which only the last, "
                                 "most conservative rung is still tried"),
    "DNN_LADDER_STARTUP": ("120", "ladder: seconds a freshly spawned child may take to its first "
                                  "heartbeat (import torch on a cold box), if above the stall"),
    "DNN_LADDER_DEADLINE": ("540", "ladder: seconds from the supervisor's start after which "
                                   "no attempt runs on (a running child is killed); the "
                                   "data-parallel comparison runs only if it fits before it"),
    "DNN_LADDER_FAULT": ("", "ladder fault injection (tests): 'rung=stage:S,step:N,kind:K;...' "
                             "-- the child of that rung gets DNN_FAULT (stage = rank)"),
    "DNN_PIPE": ("auto", "pipeline transport: auto (IPC with relays on RCCL jobs when every "
                         "GPU maps its peers, first step verified against RCCL) | rccl | ipc "
                         "(xGMI peer copies + stream flags)"),
    "DNN_IPC_RELAYS": ("auto", "ipc transport: stripe every hop over the direct link + this "
                               "many relay ranks (two-link paths; native step only); auto = "
                               "per-hop counts from the directed-link load model "
                               "(comm.relay_plan: up to 6 on 8 ranks, wide boundaries first)"),
    "DNN_IPC_VERIFY": ("auto", "verify the first IPC step bitwise against the fallback "
                               "transport: auto (with DNN_PIPE=auto) | 1 | 0"),
    "DNN_VERIFY_FLAG_TIMEOUT": ("20", "seconds a flag wait of the IPC first-step "
                                      "verification may spin before the step is declared "
                                      "stalled (steady state: DNN_FLAG_TIMEOUT, 120 s)"),
    "DNN_FAULT_IPC_VERIFY": ("", "ranks whose IPC verification step is corrupted (tests the "
                                 "fallback)"),
    "DNN_CHAIN_FUSED": ("1", "device-side chain: a stage's last (non-softmax) layer runs fused "
                             "with the hop's send (chain_gemv_send: rows straight into the "
                             "consumer's slot); 0 = gemv + chain_send"),
    "DNN_CHAIN_NATIVE": ("1", "device-side chain: rank 0 with a one-layer stage runs each request "
                              "as one native call (runtime/chain_host.cpp: H2D, layer + send, "
                              "result wait, D2H, ack, GIL-free completion spin)"),
    "DNN_CHAIN_ONE_LAUNCH": ("0", "device-side chain, one-layer stages > 0: the receive folded into "
                                  "chain_gemv_send too (one kernel per hop; every workgroup "
                                  "waits on the input flag). Opt-in: slower with several waiting "
                                  "stages on one GPU (profiles/r4_chain)"),
    "DNN_CHAIN_PERSIST": ("1", "device-side chain, one-layer stages > 0: one persistent kernel "
                               "per stage (chain_stage_run) serves every request with no host "
                               "work per request; 0 = the host enqueues each request's kernels"),
    "DNN_CHAIN_DOORBELL": ("1", "device-side chain with persistent stages: rank 0's one-layer "
                                "stage is a persistent kernel too, fed through host memory "
                                "(rows, header, flag), and the last rank writes results into a "
                                "shared host-memory ring: no HIP call per request on rank 0"),
    "DNN_CHAIN_TRACE": ("0", "device-side chain: 1 = every rank logs each request's steps and, "
                             "after synchronising, its flag words (diagnosis; serialises)"),
    "DNN_CHAIN_FAST": ("1", "rank chain: serving-size requests (<= 8 rows) take the device-side "
                            "chain (serve/fastpath.py: IPC slots + flags, no host hop); 0 = "
                            "the message-passing chain for every request"),
    "DNN_SERVE_REPLAY": ("graph", "serving engine replay: graph | native | eager"),
    "DNN_SYNC_DEBUG": ("0", "synchronise + check after every kernel (race / fault hunting)"),
    "DNN_AUTOBUILD": ("1", "build the native extension on import if it is missing"),
    "DNN_NATIVE_PATH": ("", "load the native extension from this file instead of the in-tree "
                            "build (same-box A/B of two kernel builds; bench / probes only)"),
    # multi-rank rehearsal on one GPU
    "DNN_FORCE_DEVICE": ("", "run every rank on this device (one-GPU rehearsals)"),
    "DNN_DIST_BACKEND": ("nccl", "process-group backend of bench.py (gloo for rehearsals)"),
    # serving / failure handling
    "DNN_HOP_TIMEOUT": ("10", "per-hop deadline of the stage worker (grpc_node.py:133)"),
    "DNN_FAULT": ("", "training fault injection 'stage:S,step:N,kind:crash|hang|nan|raise'"),
    "DNN_FAULT_STAGE": ("", "serving chain: rank that fails"),
    "DNN_FAULT_KIND": ("raise", "serving chain fault kind: raise | hang"),
    "DNN_FAULT_AFTER": ("0", "serving chain: requests served before the fault"),
    "DNN_WORKER_DEVICE": ("auto", "stage worker device: auto | cpu"),
}


def get(name: str, env=None) -> str:
    """The switch's value from ``env`` (default: the process environment) or its default. A
    stage worker passes the environment it was configured with (the reference's per-container
    env contract, serve/worker.py)."""
    if name not in SWITCHES:
        raise KeyError(f"undeclared switch {name}")
    return (os.environ if env is None else env).get(name, SWITCHES[name][0])


def flag(name: str) -> bool:
    return get(name) == "1"


def active() -> dict[str, str]:
    """The switches set to a non-default value in this process."""
    return {k: os.environ[k] for k in SWITCHES
            if k in os.environ and os.environ[k] != SWITCHES[k][0]}


def describe() -> str:
    return "\n".join(f"{k:24s} default {v[0]!r:10s} {v[1]}" for k, v in SWITCHES.items())
