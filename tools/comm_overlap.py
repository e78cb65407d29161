"""Overlap of the gradient exchange's RCCL kernels with the backward kernels, from a rocprofv3
kernel trace of ``bench.py --exchange`` (tools/gpu_r03_e.sh).

    python tools/comm_overlap.py KERNEL_TRACE_CSV [RCCL_API_TRACE_CSV]

For every collective kernel (RCCL: names containing "nccl" / "rccl", case-insensitive) of the last
timed steps: its stream / queue, duration, and the compute kernels whose execution intervals
intersect it (how much of the collective ran under compute, and on which other queue).

With the RCCL API trace (rocprofv3 --rccl-trace): every ncclAllReduce / ncclBroadcast call of the
last step, when the host issued it relative to that step's backward kernels -- which kernel was
executing on the GPU at the call, and how many backward kernels were still to start after it.  On
a one-rank group (bench.py --exchange on one GPU) RCCL launches no reduction kernel (an average
over one rank is the identity), so the API trace is the evidence of issue-time overlap there.
"""
import csv
import sys


def short(name):
    name = name.replace("bnn::(anonymous namespace)::", "").replace("void ", "").strip()
    if name.startswith("at::native::"):                     # torch's own kernels: functor name only
        for tag in ("FillFunctor", "CUDAFunctorOnSelf_add", "reduce_kernel", "nll_loss", "softmax", "where",
                    "copy", "mul", "div"):
            if tag in name:
                return "torch " + tag
        return "torch kernel"
    return name.split("(")[0][:60]


def is_comm(name):
    """RCCL's kernels: ncclDevKernel_* / rccl* on N ranks, oneRankReduce<FuncPreMulSum> on one rank
    (the AVG scaling of a one-rank all-reduce)."""
    n = name.lower()
    return "nccl" in n or "rccl" in n or "onerankreduce" in n


def api_report(path, comp_rows):
    """Host issue order of the last step: kernel launches and RCCL calls merged by correlation id
    (the order the host enqueued them; the collectives go to RCCL's own stream)."""
    calls = []
    rd = csv.DictReader(open(path))
    for r in rd:
        fn = r.get("Function", "")
        if "AllReduce" in fn or "Broadcast" in fn:
            calls.append((int(r["Correlation_Id"]), fn))
    print(f"{len(calls)} RCCL all-reduce / broadcast API calls in the trace")
    if not calls:
        return
    calls.sort()
    t0 = [c for c in calls if "Broadcast" in c[1]][-1][0]       # the last step's forward pre-hook
    seq = [(cid, "RCCL " + fn) for cid, fn in calls if cid >= t0]
    seq += [(cid, short(name)) for cid, name in comp_rows if cid >= t0]
    seq.sort()
    print("last step, host enqueue order (kernels on the compute stream, RCCL calls on RCCL's stream):")
    run, prev = 0, None
    for _, what in seq:
        if what == prev:
            run += 1
            continue
        if prev is not None:
            print(f"  {prev}{f'  x{run}' if run > 1 else ''}")
        prev, run = what, 1
    print(f"  {prev}{f'  x{run}' if run > 1 else ''}")
    ar = [i for i, (_, w) in enumerate(seq) if "AllReduce" in w]
    fp6 = [i for i, (_, w) in enumerate(seq) if w.startswith("gemm_fp6")]
    if ar and fp6:
        print(f"all-reduces issued before the step's last FP6 backward GEMM: "
              f"{sum(1 for i in ar if i < fp6[-1])} of {len(ar)}")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"],
                   r.get("Stream_Id", "")))
    comp_rows = [(int(r["Correlation_Id"]), r["Kernel_Name"]) for r in rows
                 if not is_comm(r["Kernel_Name"]) and "rocclr" not in r["Kernel_Name"]]
    ks.sort()
    comm = [k for k in ks if is_comm(k[2])]
    comp = [k for k in ks if k not in comm and "rocclr" not in k[2]]
    print(f"{len(comm)} collective kernel launches, {len(comp)} compute launches in the trace")
    if len(sys.argv) > 2 and sys.argv[2]:
        api_report(sys.argv[2], comp_rows)
    if not comm:
        return
    names = sorted({short(k[2]) for k in comm})
    print("collective kernels:", ", ".join(names))
    tot = under = 0
    for s, e, name, q, st in comm[-24:]:
        ov = [(max(s, s2), min(e, e2), n2, q2) for s2, e2, n2, q2, _ in comp if s2 < e and e2 > s]
        cover = sum(b - a for a, b, _, _ in ov)
        tot += e - s
        under += min(cover, e - s)
        others = sorted({short(n) for _, _, n, _ in ov})
        print(f"  {short(name):40s} queue {q} stream {st}: {(e - s) / 1e3:8.1f} us, under compute "
              f"{min(cover, e - s) / 1e3:8.1f} us  [{', '.join(others[:3])}{' ...' if len(others) > 3 else ''}]")
    print(f"last {min(24, len(comm))} collectives: {tot / 1e3:.1f} us, {under / max(tot, 1):.2%} of it overlapped "
          f"by compute kernels on other queues")


if __name__ == "__main__":
    main()
