"""The stream topology of tools/exp/capture_fork_repro.hip, captured through torch (torch.cuda.graph, torch streams,
Stream.wait_stream), to locate what the two-lane GraphedRAFT capture adds to it. The HIP-only
repro captures and replays every topology cleanly (profiles/r06/r6s2_*.log), so the crash needs something torch or
the forward does. Modes (argv[1]):
    ops     -- in-place kernels on preallocated tensors only (the HIP repro's work, through torch)
    alloc   -- every kernel out of place: each launch allocates its output from the caching allocator on the stream
               it runs on (lane / side streams included), as the forward's intermediate tensors do
    lanealloc -- in place everywhere except on the lanes' side streams (E0 after the encoders, S1), which allocate
    noside  -- ops without the lanes' side streams (graph.py's configuration)
    keep    -- ops, every fork/join event kept alive until after the capture
    raw     -- ops, captured by hipStreamBeginCapture / hipStreamEndCapture called through ctypes instead of
               torch.cuda.graph (torch does not know it is capturing; no allocation happens in this mode)
Prints "RESULT <mode> ok replay_equal=<0|1>" or dies in capture_end.
    python -X faulthandler tools/exp/capture_fork_torch_repro.py alloc
"""
import sys

import torch


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "ops"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    dev = torch.device("cuda", 0)
    streams = {}

    def side_stream(slot):  # model/update.py _side_stream: keyed by (owner stream, slot)
        key = (torch.cuda.current_stream(dev).stream_id, slot)
        if key not in streams:
            streams[key] = torch.cuda.Stream(device=dev)
        return streams[key]

    buf = torch.zeros(4096, device=dev)
    kept = []

    def wait_stream(consumer, producer):  # torch.cuda.Stream.wait_stream, optionally keeping the event alive
        ev = producer.record_event()
        consumer.wait_event(ev)
        if mode == "keep":
            kept.append(ev)
    slot = [0]

    def k(n=1, alloc=False):
        for _ in range(n):
            i = slot[0] % 4096
            slot[0] += 1
            if alloc:
                # fresh allocations on the current stream, dropped at once (freed back to that stream's pool)
                buf[i : i + 1].copy_(buf[i : i + 1] * 0.5 + float(i))
            else:
                buf[i : i + 1].mul_(0.5).add_(float(i))

    a_all = mode == "alloc"

    def forward():
        slot[0] = 0
        C = torch.cuda.current_stream(dev)
        E0, E1 = side_stream(0), side_stream(1)
        k(2, a_all)
        wait_stream(E1, C)
        with torch.cuda.stream(E1):
            k(12, a_all)
        k(3, a_all)
        wait_stream(E0, C)
        with torch.cuda.stream(E0):
            k(12, a_all)
        k(12, a_all)
        wait_stream(C, E1)
        k(1, a_all)
        wait_stream(C, E0)
        k(5, a_all)
        L1 = side_stream(101)
        wait_stream(L1, C)
        with torch.cuda.stream(L1):
            S1 = side_stream(201)
            k(3, a_all)
        S0 = side_stream(0)  # owner C, slot 0: the encoders' E0
        side_alloc = a_all or mode == "lanealloc"
        for it in range(iters):
            last = it == iters - 1
            if last:
                wait_stream(L1, C)
            for lane, side in ((C, S0), (L1, S1)):
                with torch.cuda.stream(lane):
                    if mode == "noside":
                        k(5)
                    else:
                        wait_stream(side, lane)
                        with torch.cuda.stream(side):
                            k(3, side_alloc)
                        k(2, a_all)
                        wait_stream(lane, side)
                    k(8, a_all)
            if last:
                wait_stream(C, L1)
                k(1, a_all)
        wait_stream(C, L1)
        k(1, a_all)

    forward()
    torch.cuda.synchronize()
    ref = buf.clone()
    print("eager ok", flush=True)
    cap = torch.cuda.Stream(device=dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):
        buf.zero_()
        forward()  # warm-up on the capture stream: its side streams are the ones the capture uses
    torch.cuda.current_stream(dev).wait_stream(cap)
    torch.cuda.synchronize()
    if mode == "raw":
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        graph, exe = ctypes.c_void_p(), ctypes.c_void_p()
        sp = ctypes.c_void_p(cap.cuda_stream)
        with torch.cuda.stream(cap):
            assert hip.hipStreamBeginCapture(sp, 0) == 0  # hipStreamCaptureModeGlobal
            forward()
            print("calling hipStreamEndCapture", flush=True)
            rc = hip.hipStreamEndCapture(sp, ctypes.byref(graph))
        print("end capture rc", rc, flush=True)
        assert rc == 0
        assert hip.hipGraphInstantiate(ctypes.byref(exe), graph, None, None, ctypes.c_size_t(0)) == 0
        buf.zero_()
        torch.cuda.synchronize()
        assert hip.hipGraphLaunch(exe, sp) == 0
    else:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            forward()
        print("captured", flush=True)
        buf.zero_()
        g.replay()
    torch.cuda.synchronize()
    print(f"RESULT {mode} ok replay_equal={int(torch.equal(buf, ref))}", flush=True)


if __name__ == "__main__":
    main()
