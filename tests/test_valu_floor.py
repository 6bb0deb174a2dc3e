"""CPU: tools/valu_floor.py, the VALU roofline of the long double folds
(DESIGN.md section 4), on this build's code object: the per-element stream
is found, every opcode is priced, and the build's lib/valu_floor.json (what
bench.py reports) is the same computation."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
OBJ = os.path.join(ROOT, "osss-gasnet_amd", "lib", "combine_t_longdouble.o")
RATES = os.path.join(ROOT, "profiles", "r04", "valu", "valu_rate.jsonl")
FLOOR = os.path.join(ROOT, "osss-gasnet_amd", "lib", "valu_floor.json")


@pytest.mark.skipif(not os.path.exists(OBJ), reason="library not built")
def test_valu_floor_of_the_long_double_legs():
    import valu_floor
    built = json.load(open(FLOOR))
    for leg, (sub, n, stores) in valu_floor.BENCH_LEGS.items():
        fl = valu_floor.floor(OBJ, sub, RATES, n, stores)
        assert fl == built[leg], leg
        assert sum(fl["by_kind"].values()) == fl["valu_per_element_wave"] > 500, fl
        # every kind priced has a measured rate; half-rate kinds are a real share of an x87 chain
        rates = {json.loads(ln)["kind"] for ln in open(RATES)}
        assert set(fl["by_kind"]) <= rates, fl["by_kind"]
        assert fl["by_kind"]["v_add_u32"] < fl["valu_per_element_wave"], fl
        assert 20 < fl["floor_us"] < 400, fl
    # the sum's additions cost more than the product's multiplications
    assert built["rs_shard_n8_longdouble_sum"]["floor_us"] > built["rs_shard_n8_longdouble_prod"]["floor_us"]
