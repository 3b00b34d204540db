"""Dump fnet (split S32 rows) and cnet outputs of the split encoders for 8 Sintel images, with the library this process
loads (OFLOW_LIB), to gpurun_out/enc_<TAG>.pt; `python tools/exp/enc_dump.py --compare A B` reports whether two dumps
are bit-identical (max |d| otherwise). Used to check that an encoder kernel change keeps the outputs bit-identical."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def compare(a, b):
    x = torch.load(os.path.join(REPO, "gpurun_out", f"enc_{a}.pt"), weights_only=True)
    y = torch.load(os.path.join(REPO, "gpurun_out", f"enc_{b}.pt"), weights_only=True)
    for k in x:
        same = torch.equal(x[k], y[k])
        d = 0.0 if same else float((x[k].float() - y[k].float()).abs().max())
        print(f"{k}: bit_identical={same} max|d|={d:.3e}")


def main():
    from model import RAFT, synthetic
    from model.extractor import SplitEncoder

    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    img0, _ = synthetic.synthetic_pair(8, 440, 1024, seed=0)
    x = (2 * (img0.to(dev) / 255.0) - 1.0).contiguous()
    out = {}
    with torch.inference_mode():
        out["fnet"] = SplitEncoder(model.fnet)(x, split_out=True, stem_from_image=True).cpu()
        out["cnet"] = SplitEncoder(model.cnet)(x, stem_from_image=True).cpu()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    torch.save(out, os.path.join(REPO, "gpurun_out", f"enc_{os.environ.get('TAG', 'x')}.pt"))
    print("saved", {k: tuple(v.shape) for k, v in out.items()})


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        main()
