"""CPU: the DIN host encoder (nrk.rank.din) reproduces DINDataset.__getitem__
+ collate_fn (src/rank/DIN.py:289-520) exactly on the reference-generated
fixture tests/golden/din_encode_small.npz -- both the float-row case (ids
upcast to float, user/item/history features all encode to 0) and the
object-row case (ids found)."""
import numpy as np
import pandas as pd
import pytest


class _Enc:
    def __init__(self, classes):
        self.classes_ = classes


@pytest.mark.parametrize("case", ["out", "obj"])
def test_encoder_matches_reference(golden, case):
    from nrk.rank.din import encode_samples, iloc_columns

    g = golden("din_encode_small")
    uf = [k.split("::")[1] for k in g.files if k.startswith("classes::")]
    nu, ni = g["prof_vals"].shape[1], g["ifeat_vals"].shape[1]
    user_f, item_f, ctx_f = uf[:nu], uf[nu:nu + ni], uf[nu + ni:]
    enc = {f: _Enc(g[f"classes::{f}"]) for f in uf}
    upd = {str(u): {f: float(v) for f, v in zip(user_f, row)}
           for u, row in zip(g["prof_users"], g["prof_vals"])}
    ifd = {str(i): {f: int(v) for f, v in zip(item_f, row)}
           for i, row in zip(g["ifeat_items"], g["ifeat_vals"])}
    off = g["hist_offsets"]
    uhd = {str(u): [str(x) for x in g["hist_items"][off[n]:off[n + 1]]]
           for n, u in enumerate(g["hist_users"])}
    df = pd.DataFrame({"user_id": g["main_user"], "item_id": g["main_item"], "label": g["main_label"]})
    for n, f in enumerate(ctx_f):
        df[f] = g["main_ctx"][:, n]
        if case == "obj":
            df[f] = df[f].astype(str)
    cols = iloc_columns(df, ["user_id", "item_id"] + ctx_f)
    out = encode_samples(cols["user_id"], cols["item_id"], cols, upd, ifd, uhd,
                         user_f, item_f, ctx_f, enc, int(g["T"]))
    for k in ("user", "item", "hist", "ctx", "mask"):
        assert np.array_equal(out[k], g[f"{case}_{k}"]), k
