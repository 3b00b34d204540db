"""Debug: RAFT pair lanes with per-lane lookups, lookup through (a) torch.ops.oflow (product) or (b) the C ABI via
ctypes on torch.cuda.current_stream(); repeated runs vs the single-lane result."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)
import torch
from model import RAFT, synthetic
from optical_flow import _native as N
DEV = torch.device("cuda", 0)
mode = sys.argv[1] if len(sys.argv) > 1 else "ops"
if mode == "ctypes":
    def nhwc(pyr, coords, radius, out):
        lib = N.load()
        b, _, h, w = coords.shape
        nl = len(pyr.levels)
        ptrs = (ctypes.c_void_p * nl)(*[t.data_ptr() for t in pyr.levels])
        hs = (ctypes.c_int * nl)(*[d[0] for d in pyr.dims])
        ws = (ctypes.c_int * nl)(*[d[1] for d in pyr.dims])
        st = lib.oflow_corr_lookup_tiled_nhwc_f32(ptrs, hs, ws, nl, coords.data_ptr(), b, h, w, int(radius), out.data_ptr(),
                                                 int(out.shape[1]), ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream))
        assert st == 0
        return out
    N.corr_lookup_tiled_nhwc = nhwc
elif mode == "canonpersist":
    # canonical pyramid materialised ONCE on the main stream (untile), lanes' lookups read slices of it concurrently
    CANON = {}
    def nhwc(pyr, coords, radius, out):
        b, _, h, w = coords.shape
        if id(pyr) not in CANON:
            CANON[id(pyr)] = [pyr.untile(l) for l in range(len(pyr.levels))]
        o = N.corr_lookup(CANON[id(pyr)], coords, radius)
        out.view(b, h, w, -1).copy_(o.permute(0, 2, 3, 1))
        return out
    N.corr_lookup_tiled_nhwc = nhwc
    import model.corr as MC
    orig_bs = MC.CorrBlock.batch_slice
    FULL = {}
    def batch_slice(self, b0, b1):
        v = orig_bs(self, b0, b1)
        if id(self) not in FULL:
            FULL.clear()
            FULL[id(self)] = [self._tiled.untile(l) for l in range(len(self._tiled.levels))]  # main stream
        hw = self._tiled.dims[0][0] * self._tiled.dims[0][1]
        CANON[id(v._tiled)] = [t[b0 * hw : b1 * hw] for t in FULL[id(self)]]
        return v
    MC.CorrBlock.batch_slice = batch_slice
elif mode in ("nchw", "canon"):
    # the same rows through the NCHW tiled kernel (v5, OUT=0) or the canonical-layout kernel, permuted on the stream
    def nhwc(pyr, coords, radius, out):
        b, _, h, w = coords.shape
        if mode == "nchw":
            o = N.corr_lookup_tiled(pyr, coords, radius)
        else:
            o = N.corr_lookup([pyr.untile(l) for l in range(len(pyr.levels))], coords, radius)
        out.view(b, h, w, -1).copy_(o.permute(0, 2, 3, 1))
        return out
    N.corr_lookup_tiled_nhwc = nhwc
elif mode == "check":
    orig = N.corr_lookup_tiled_nhwc
    LOG = []
    def nhwc(pyr, coords, radius, out):
        snap = coords.clone()            # on this lane's stream, right before the lookup
        r = orig(pyr, coords, radius, out)
        LOG.append((pyr, snap, radius, out.clone()))  # the rows as written, copied on the same stream
        return r
    N.corr_lookup_tiled_nhwc = nhwc
elif mode in ("ownbefore", "otherbefore"):
    orig = N.corr_lookup_tiled_nhwc
    from model.update import _SIDE_STREAMS
    def nhwc(*a):
        cur = torch.cuda.current_stream(DEV)
        if mode == "ownbefore":
            cur.synchronize()  # this lane's stream only (host waits)
        else:
            # every other stream (main, lanes, side streams) finished what it has enqueued so far
            for st in [torch.cuda.default_stream(DEV)] + list(_SIDE_STREAMS.values()):
                if st != cur:
                    st.synchronize()
        return orig(*a)
    N.corr_lookup_tiled_nhwc = nhwc
elif mode in ("before", "after", "streamafter"):
    orig = N.corr_lookup_tiled_nhwc
    def nhwc(*a):
        if mode == "before":
            torch.cuda.synchronize()
        r = orig(*a)
        if mode == "after":
            torch.cuda.synchronize()
        if mode == "streamafter":
            torch.cuda.current_stream(DEV).synchronize()
        return r
    N.corr_lookup_tiled_nhwc = nhwc
elif mode == "sync":
    orig = N.corr_lookup_tiled_nhwc
    def nhwc(*a):
        torch.cuda.synchronize()
        r = orig(*a)
        torch.cuda.synchronize()
        return r
    N.corr_lookup_tiled_nhwc = nhwc
m = RAFT().eval(); m.load_state_dict(synthetic.synthetic_state_dict(m.state_dict())); m = m.to(DEV)
img0, img1 = synthetic.synthetic_pair(2, 128, 160, seed=5)
b = 8
p0 = img0.repeat(4, 1, 1, 1)[:b].to(DEV); p1 = img1.repeat(4, 1, 1, 1)[:b].to(DEV)
p1[-1] = torch.roll(p1[-1], 3, dims=-1)
bad = 0
with torch.inference_mode():
    m.pair_lanes, m.pair_lookup = 1, "joined"
    ref, _ = m(p0, p1, iters=4, test_mode=True)
    ref = ref.clone()
    m.pair_lanes, m.pair_lookup = 2, "lane"
    for _ in range(8):
        lo, _ = m(p0, p1, iters=4, test_mode=True)
        bad += int(not torch.equal(lo, ref))
print(mode, "mismatching runs", bad, "of 8", flush=True)
if mode == "check":
    torch.cuda.synchronize()
    nbad = 0
    for pyr, snap, radius, rows in LOG:
        again = torch.empty_like(rows)
        orig(pyr, snap, radius, again)
        torch.cuda.synchronize()
        if not torch.equal(again, rows):
            nbad += 1
            if nbad <= 4:
                d = (again != rows)
                qi, ci = torch.nonzero(d, as_tuple=True)
                print("  rows", rows.shape[0], "diff elems", int(d.sum()), "queries", sorted(set(qi.tolist()))[:12],
                      "n_queries", len(set(qi.tolist())), "channels", sorted(set(ci.tolist()))[:20],
                      "levels", sorted(set((ci // 81).tolist())),
                      "sample got/ref", [(float(rows[a, b]), float(again[a, b])) for a, b in list(zip(qi.tolist(), ci.tolist()))[:3]])
    print("lookups whose rows differ from a quiet recompute on the same coords:", nbad, "of", len(LOG))
