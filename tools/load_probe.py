import os, sys, time, json
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import util, sc_polar_decoder_hls_amd as pkg, torch
for sw in sys.argv[1].split(","):
    os.environ["POLAR_SC_SUB_WORDS"] = sw
    d = pkg.Decoder(util.mask(sys.argv[2]))
    t = time.time()
    d.compile()
    tc = time.time() - t
    try:
        d.prepare(512)
        ok = True; err = ""
    except Exception as e:
        ok = False; err = str(e)
    print(json.dumps({"sub_words": sw, "kinds": d.stats["n_sub_kinds"], "compile_s": round(tc, 1), "load_ok": ok, "err": err[:200]}), flush=True)
