"""CPU-baseline calibration (build container only, never on the GPU box): time the reference's
own align() (imported from /root/reference behind the SURVEY.md §8(c) stand-ins, as
tests/golden/make_golden.py does) against bench.py's reference-structured CPU path
(_cpu_reference_align: CPU forward + oracle TorchPort DP + host aggregation) on identical
inputs: the same random-weight wav2vec2-base, the same 30 s clip and transcript, device='cpu',
at 1 and at os.cpu_count() threads.  Also the DP alone: reference get_trellis/backtrack/
merge_repeats vs TorchPort.  Prints one JSON line; the numbers go to BASELINE.md."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
import make_golden  # noqa: E402  (stand-ins + reference loader)
import torch  # noqa: E402

import bench  # noqa: E402
from oracle.oracle import TorchPort  # noqa: E402
from whisperx_amd import synthetic  # noqa: E402


def best(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    A, _V, _pc = make_golden._load_reference()
    segs, audio = bench._e2e_inputs(1, 11)
    dictionary = synthetic.w2v_dictionary()
    meta = {"language": "en", "dictionary": dictionary, "type": "huggingface"}
    out = {"host": os.uname().machine, "cpu_count": os.cpu_count()}
    for threads in (1, os.cpu_count()):
        torch.set_num_threads(threads)
        model = bench._w2v_base("cpu", 11)
        ref = lambda: A.align([dict(s) for s in segs], model, meta, audio.numpy(), "cpu")  # noqa: E731
        port = lambda: bench._cpu_reference_align(segs, model, dictionary, audio[None])  # noqa: E731
        ref(), port()
        r, p = best(ref, 3), best(port, 3)
        out[f"align_threads{threads}"] = {"reference_s": r, "port_s": p, "port_over_reference": p / r}
    # DP alone on the clip's emission
    torch.set_num_threads(1)
    with torch.inference_mode():
        em = torch.log_softmax(model(audio[None]).logits, -1)[0]
    seg = dict(segs[0])
    from whisperx_amd import alignment as W
    W._prepare(seg, dictionary, "en")
    toks = [dictionary[c] for c in "".join(seg["clean_char"])]
    tp = TorchPort()

    def ref_dp():
        tr = A.get_trellis(em, toks, 0)
        path = A.backtrack(tr, em, toks, 0)
        return A.merge_repeats(path, "".join(seg["clean_char"]))

    r, p = best(ref_dp, 3), best(lambda: tp.align_dp(em, toks, 0), 3)
    out["dp_threads1"] = {"T": int(em.shape[0]), "N": len(toks), "reference_s": r, "port_s": p,
                          "port_over_reference": p / r}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
