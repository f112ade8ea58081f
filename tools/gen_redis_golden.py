"""Collect the RESP request vectors of the reference's own parser tests
(test_redis_parse_req_success, /root/reference/src/test_all.c:109-230) into
tests/golden/redis_req_cases.json: each request's bytes and the MSG_REQ_REDIS_*
type the reference asserts for it. Data only; run here, where the reference is."""
import ast
import json
import os
import re
import sys

SRC = "/root/reference/src/test_all.c"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "redis_req_cases.json")


def main() -> None:
    text = open(SRC).read()
    body = text[text.index("static void test_redis_parse_req_success(void)"):]
    body = body[:body.index("\n}\n")]
    cases = []
    for m in re.finditer(r'test_redis_parse_req_success_case\(((?:\s*"(?:[^"\\]|\\.)*")+)\s*,\s*MSG_REQ_REDIS_(\w+)\)',
                         body):
        lits = re.findall(r'"((?:[^"\\]|\\.)*)"', m.group(1))
        req = "".join(ast.literal_eval('"' + s + '"') for s in lits)
        cases.append({"req": req, "type": m.group(2)})
    json.dump({"source": "src/test_all.c:109-230 (test_redis_parse_req_success)", "cases": cases},
              open(OUT, "w"), indent=0)
    print(len(cases), "cases ->", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
