"""Debug: split vs single decode on the golden decode inputs, per size."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpoporon_amd as P
g = np.load("tests/golden/rs255_golden.npz")
os.environ["POPORON_AMD_DECODE_PATH"] = "split"
hs = P.Poporon.default()
os.environ["POPORON_AMD_DECODE_PATH"] = "single"
h1 = P.Poporon.default()
sizes = g["dec_size"]
for s in np.unique(sizes):
    sel = np.nonzero(sizes == s)[0]
    s = int(s)
    a = hs.decode_batch(g["dec_in"][sel, :s], g["dec_in"][sel, s:s + 32])
    b = h1.decode_batch(g["dec_in"][sel, :s], g["dec_in"][sel, s:s + 32])
    bad = np.nonzero((a[0] != b[0]) | (a[1] != b[1]) | (np.concatenate([a[2], a[3]], 1) != np.concatenate([b[2], b[3]], 1)).any(1))[0]
    print("size", s, "n", len(sel), "mismatch", len(bad), "split ok/cor", a[0][bad[:6]], a[1][bad[:6]], "single", b[0][bad[:6]], b[1][bad[:6]])
    if len(bad):
        # how many errors do the bad ones carry?
        i = sel[bad[:6]]
        diff = (g["dec_in"][i, :s + 32] != g["dec_out"][i, :s + 32]).sum(1)
        print("   errors in bad:", diff, "golden ok", g["dec_ok"][i], "cor", g["dec_cor"][i])
