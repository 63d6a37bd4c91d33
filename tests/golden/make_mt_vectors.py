"""Generate tests/golden/mt_vectors.json from CPython's own stdlib `random`.

These vectors pin the oracle's and the device kernel's MT19937 restatement
(CPython 3.10 semantics: random.seed(int), getrandbits(32), random(),
_randbelow via randrange/randint, sample(pop, 1)). They come from the Python
standard library only, never from the reference.
Run: python tests/golden/make_mt_vectors.py
"""
import json
import os
import random
import sys

SEEDS = [0, 1, 2, 42, 12345, 2**32 - 1, 2**32, 2**40 + 7, 2**63 + 5]


def main():
    out = {"python": sys.version.split()[0], "cases": []}
    for seed in SEEDS:
        r = random.Random(seed)
        state = list(r.getstate()[1])
        case = {"seed": seed, "state_words_head": state[:8], "state_index": state[624]}
        case["genrand"] = [r.getrandbits(32) for _ in range(700)]  # crosses one twist
        r = random.Random(seed)
        case["random"] = [r.random().hex() for _ in range(50)]
        r = random.Random(seed)
        # randbelow via randrange(n) for assorted n, interleaved (rejection paths)
        ns = [1, 2, 3, 5, 7, 8, 13, 25, 97, 100, 1000, 2**31 + 1]
        case["randbelow_n"] = ns * 5
        case["randbelow"] = [r.randrange(n) for n in ns * 5]
        r = random.Random(seed)
        case["sample1_n"] = [1, 2, 3, 4, 24, 25, 30, 96] * 4
        case["sample1"] = [r.sample(list(range(n)), 1)[0] for n in case["sample1_n"]]
        r = random.Random(seed)
        case["randint_ab"] = [[0, 7], [0, 2], [0, 0], [0, 31], [3, 9]] * 4
        case["randint"] = [r.randint(a, b) for a, b in case["randint_ab"]]
        out["cases"].append(case)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mt_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", path)


if __name__ == "__main__":
    main()
