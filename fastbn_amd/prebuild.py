"""Prebuild plan-specialized JT kernels into the in-tree code-object cache (fastbn_amd/kcache).

The cache key is a hash of the generated source and the compile options, so a kernel built here
is found by any process that plans the same network (jt_jit.hip); a miss compiles with hiprtc at
first run instead.
"""
import os
import tempfile

from . import api, synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALARM_XML = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
# eligible synthetic network used by the GPU parity tests (tests/test_gpu_jt.py)
SYNTH_SMALL = dict(n=60, seed=5, window=6)


def synth_small_xml(dirname):
    path = os.path.join(dirname, "synth60.xml")
    synth.random_network(SYNTH_SMALL["n"], seed=SYNTH_SMALL["seed"], window=SYNTH_SMALL["window"], path=path)
    return path


def prebuild(xml_paths, layouts=(0,)):
    out = []
    for xml in xml_paths:
        jt = api.JunctionTree(api.Network(xml), device=-1)
        if jt.info["specialized_eligible"]:
            for layout in layouts:  # output layouts (0 case-major, 1 variable-major: bench.py's ALARM)
                jt.set_output_layout(layout)
                for exact in (None, True):  # both arithmetic orders (default fast, exact on request)
                    jt.set_exact(exact)
                    out.append(jt.build_kernel())
    return out


def fixture_xmls(dirname):
    """The XMLBIF fixtures of the GPU tests (tests/golden/synth_nets/*.xml.gz), unpacked."""
    import glob
    import gzip
    out = []
    for gz in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "synth_nets", "*.xml.gz"))):
        path = os.path.join(dirname, os.path.basename(gz)[:-3])
        with gzip.open(gz, "rb") as f, open(path, "wb") as g:
            g.write(f.read())
        out.append(path)
    return out


# code-generation options the GPU tests run ALARM under (tests/test_gpu_jt_fast.py)
ALARM_TEST_OPTIONS = ({"FBN_JT_LEAF_RC": "1"}, {"FBN_JT_LDS_POOL": "0"}, {"FBN_JT_MARG_V2": "0"})


def prebuild_options(xml, options):
    """The fast-order kernel of `xml` under each set of generator environment options (read when
    the kernel is generated), built in a child process per set."""
    import subprocess
    import sys
    out = []
    for opt in options:
        env = dict(os.environ, **opt)
        code = ("import sys; sys.path.insert(0, %r); from fastbn_amd import api; "
                "print(api.JunctionTree(api.Network(%r), device=-1).build_kernel())" % (REPO, xml))
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
        out.append(r.stdout.strip().splitlines()[-1])
    return out


def prebuild_default(clean=True):
    """Every eligible benchmark / test network, both orders (cache hits are free), and the ALARM
    option variants the tests use; clean: then drop the code objects no current plan uses (older
    generator versions)."""
    with tempfile.TemporaryDirectory() as d:
        built = prebuild([ALARM_XML], layouts=(0, 1)) + prebuild([synth_small_xml(d)] + fixture_xmls(d))
    built += prebuild_options(ALARM_XML, ALARM_TEST_OPTIONS)
    if clean:
        keep = {os.path.basename(p) for p in built}
        kdir = os.path.join(REPO, "fastbn_amd", "kcache")
        for f in os.listdir(kdir) if os.path.isdir(kdir) else []:
            if f.endswith(".hsaco") and f not in keep:
                os.remove(os.path.join(kdir, f))
    return built
