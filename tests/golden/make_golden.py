"""Regenerate tests/golden/ from the reference's stored DATA (run in the dev container only).

Reads (as text/JSON data, never executing reference code):
  /root/reference/HD155358.vels                                    -> HD155358.vels (copy)
  /root/reference/plotArchive/Ben's 2-1/TEST_2-1_COMPACT.vels      -> TEST_2-1_COMPACT.vels (copy)
  /root/reference/(Ex)HD155358.ipynb  cell 4 stdout (raw lines 82-97)  -> G1 vectors
                                      cell 5 stdout (line 149)          -> G2 logp
                                      cell 19 stdout (lines 717-720)    -> G4 logp + params
  /root/reference/plotArchive/Ben's 2-1/log_Ben-2-1 line 4          -> G3 curve (1000 t, 1000 rv)
                                                     RDMGHOSTS lines -> G5: the RV curves (same
      1000 times) of 45 states drawn from the second half of the reference's SMALA chain on
      TEST_2-1_COMPACT.vels (mcmc_benchmark_smala.py:79-85 writes them): posterior samples
and writes golden.json + g3_curve.npz + g5_ghosts.npz.  SURVEY.md App. B documents G1-G4.
"""
import json
import os
import shutil

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def cell_stdout(nb, idx):
    c = nb["cells"][idx]
    return "".join("".join(o.get("text", "")) for o in c.get("outputs", []) if o.get("name") == "stdout")


def main():
    shutil.copy(os.path.join(REF, "HD155358.vels"), os.path.join(HERE, "HD155358.vels"))
    shutil.copy(os.path.join(REF, "plotArchive", "Ben's 2-1", "TEST_2-1_COMPACT.vels"),
                os.path.join(HERE, "TEST_2-1_COMPACT.vels"))
    nb = json.load(open(os.path.join(REF, "(Ex)HD155358.ipynb")))
    # locate cells by content (robust to cell renumbering)
    src = ["".join(c["source"]) for c in nb["cells"]]
    i_plot = next(i for i, s in enumerate(src) if "inLinePlotObs(initial_state" in s)
    i_logp = next(i for i, s in enumerate(src) if s.strip() == "print initial_state.get_logp(obs)")
    i_best = next(i for i, s in enumerate(src) if "np.max(sm_bundle.mcmc_chainlogp)" in s)
    i_sol = next(i for i, s in enumerate(src) if s.startswith("sol = ["))
    sol = [float(x) for x in src[i_sol].split("[", 1)[1].split("]")[0].replace("\n", " ").split(",")]
    out = cell_stdout(nb, i_plot).splitlines()
    vecs = [json.loads(l) for l in out[2:14]]
    star_vx_print = float(out[15])
    g2 = float(cell_stdout(nb, i_logp).strip())
    best = cell_stdout(nb, i_best).split("\n", 1)
    g4_logp = float(best[0])
    g4_params = [float(v) for v in best[1].split("]")[0].replace("[", " ").split()]
    # G3
    lines = open(os.path.join(REF, "plotArchive", "Ben's 2-1", "log_Ben-2-1")).read().splitlines()
    vals = np.array([float(v) for v in lines[3].split()])
    assert vals.size == 2000
    np.savez(os.path.join(HERE, "g3_curve.npz"), t=vals[:1000], rv=vals[1000:])
    # G5: posterior RV curves of the reference's SMALA run (the line after each RDMGHOSTS tag)
    ghosts = [np.array([float(v) for v in lines[i + 1].split()]) for i, l in enumerate(lines)
              if l.strip() == "RDMGHOSTS"]
    assert len(ghosts) == 45 and all(g.size == 2000 and np.array_equal(g[:1000], vals[:1000]) for g in ghosts)
    np.savez_compressed(os.path.join(HERE, "g5_ghosts.npz"), t=vals[:1000], rv=np.array([g[1000:] for g in ghosts]))
    golden = {
        "G1": {
            "source": "(Ex)HD155358.ipynb:82-97 (cell %d stdout)" % i_plot,
            "planets": [{"m": sol[3], "a": sol[0], "h": sol[1], "k": sol[2], "l": sol[4]},
                        {"m": sol[8], "a": sol[5], "h": sol[6], "k": sol[7], "l": sol[9]}],
            "note": "per body: [vx,vy,vz] then [x,y,z]; first 6 before move_to_com (heliocentric), "
                    "next 6 after (barycentric); star vx printed with 12 digits",
            "helio_v": [vecs[0], vecs[2], vecs[4]], "helio_x": [vecs[1], vecs[3], vecs[5]],
            "bary_v": [vecs[6], vecs[8], vecs[10]], "bary_x": [vecs[7], vecs[9], vecs[11]],
            "star_vx_print": star_vx_print,
        },
        "G2": {"source": "(Ex)HD155358.ipynb:149 (cell %d stdout)" % i_logp, "logp_print12": g2,
               "obs": "HD155358.vels", "Npoints": 100, "hillRadiusFactor": 2.0,
               "sol": sol, "sol_order": "a0,h0,k0,m0,l0,a1,h1,k1,m1,l1 (Python 2 dict order)"},
        "G3": {"source": "plotArchive/Ben's 2-1/log_Ben-2-1:4", "state_source": "mcmc_benchmark_smala.py:32 (the first, commented-out true_state)",
               "planets": [{"m": 0.92e-3, "a": 0.2275, "h": -0.06, "k": 0.015, "l": -1.0},
                           {"m": 1.95e-3, "a": 0.3665, "h": 0.02, "k": 0.0, "l": 2.1}],
               "obs": "TEST_2-1_COMPACT.vels", "Npoints": 100, "file": "g3_curve.npz",
               "note": "STARTSTATE = get_rv_plotting(obs): 1000 times linspace(tb[0], tf[-1]) then 1000 RVs, "
                       "printed with 12 significant digits"},
        "G4": {"source": "(Ex)HD155358.ipynb:717-720 (cell %d stdout)" % i_best, "logp_print": g4_logp,
               "params_9sig": g4_params, "order": "a0,h0,k0,m0,l0,a1,h1,k1,m1,l1", "obs": "HD155358.vels",
               "Npoints": 100},
    }
    json.dump(golden, open(os.path.join(HERE, "golden.json"), "w"), indent=1)
    print("wrote golden.json, g3_curve.npz, 2 .vels files")


if __name__ == "__main__":
    main()
