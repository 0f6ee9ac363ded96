"""Writes tests/golden/*.json: the reference's own test vectors for pkg/sat,
transcribed by hand (the reference is Go and cannot run in this pipeline).

Sources (all under /root/reference):
  * TestSolve                pkg/sat/solve_test.go:97-297 (19 cases; installed ids
                             sorted, NotSatisfiable sorted as in :316-343)
  * TestNotSatisfiableError  pkg/sat/solve_test.go:46-81
  * TestDuplicateIdentifier  pkg/sat/solve_test.go:359-365
  * TestSearch               pkg/sat/search_test.go:43-66 (scripted FakeS)
  * TestOrder                pkg/sat/constraints_test.go:17-36
  * README example           README.md:38-101 (config 1; the encoding is ours,
                             README gives none)
Constraint strings: constraints.go:57,81,108,110-114,145,173-177.

Run:  python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def M():
    return {"kind": "mandatory"}


def P():
    return {"kind": "prohibited"}


def D(*ids):
    return {"kind": "dependency", "ids": list(ids)}


def C(i):
    return {"kind": "conflict", "ids": [i]}


def A(n, *ids):
    return {"kind": "atmost", "n": n, "ids": list(ids)}


def V(i, *cons):
    return {"id": i, "constraints": list(cons)}


def cstr(subject, c):
    k = c["kind"]
    if k == "mandatory":
        return "%s is mandatory" % subject
    if k == "prohibited":
        return "%s is prohibited" % subject
    if k == "dependency":
        if not c["ids"]:
            return "%s has a dependency without any candidates to satisfy it" % subject
        return "%s requires at least one of %s" % (subject, ", ".join(c["ids"]))
    if k == "conflict":
        return "%s conflicts with %s" % (subject, c["ids"][0])
    if k == "atmost":
        return "%s permits at most %d of %s" % (subject, c["n"], ", ".join(c["ids"]))
    raise ValueError(k)


def unsat(variables, applied):
    """applied: list of (var id, constraint index) in the test's sorted order."""
    by = {v["id"]: v for v in variables}
    strs = [cstr(v, by[v]["constraints"][ci]) for v, ci in applied]
    return {"type": "NotSatisfiable", "applied": [{"var": v, "constraint": ci} for v, ci in applied],
            "string": "constraints not satisfiable: " + ", ".join(strs)}


def testsolve():
    cases = []

    def case(name, variables, installed=None, error=None, line=None):
        cases.append({"name": name, "line": line, "variables": variables,
                      "installed": installed, "error": error})

    case("no variables", [], line=98)
    case("unnecessary variable is not installed", [V("a")], line=101)
    case("single mandatory variable is installed", [V("a", M())], ["a"], line=105)
    vs = [V("a", M(), P())]
    case("both mandatory and prohibited produce error", vs,
         error=unsat(vs, [("a", 0), ("a", 1)]), line=110)
    case("dependency is installed", [V("a"), V("b", M(), D("a"))], ["a", "b"], line=124)
    case("transitive dependency is installed",
         [V("a"), V("b", D("a")), V("c", M(), D("b"))], ["a", "b", "c"], line=132)
    case("both dependencies are installed",
         [V("a"), V("b"), V("c", M(), D("a"), D("b"))], ["a", "b", "c"], line=141)
    case("solution with first dependency is selected",
         [V("a"), V("b", C("a")), V("c", M(), D("a", "b"))], ["a", "c"], line=150)
    case("solution with only first dependency is selected",
         [V("a"), V("b"), V("c", M(), D("a", "b"))], ["a", "c"], line=159)
    case("solution with first dependency is selected (reverse)",
         [V("a"), V("b", C("a")), V("c", M(), D("b", "a"))], ["b", "c"], line=168)
    vs = [V("a", M()), V("b", M(), C("a"))]
    case("two mandatory but conflicting packages", vs,
         error=unsat(vs, [("a", 0), ("b", 0), ("b", 1)]), line=177)
    case("irrelevant dependencies don't influence search Order",
         [V("a", D("x", "y")), V("b", M(), D("y", "x")), V("x"), V("y")], ["b", "y"], line=198)
    vs = [V("a", M(), D("x", "y"), A(1, "x", "y")), V("x", M()), V("y", M())]
    case("cardinality constraint prevents resolution", vs,
         error=unsat(vs, [("a", 2), ("x", 0), ("y", 0)]), line=208)
    case("cardinality constraint forces alternative",
         [V("a", M(), D("x", "y"), A(1, "x", "y")), V("b", M(), D("y")), V("x"), V("y")],
         ["a", "b", "y"], line=230)
    case("two dependencies satisfied by one variable",
         [V("a", M(), D("y")), V("b", M(), D("x", "y")), V("x"), V("y")], ["a", "b", "y"], line=240)
    case("foo two dependencies satisfied by one variable",
         [V("a", M(), D("y", "z", "m")), V("b", M(), D("x", "y")), V("x"), V("y"), V("z"), V("m")],
         ["a", "b", "y"], line=250)
    case("result size larger than minimum due to preference",
         [V("a", M(), D("x", "y")), V("b", M(), D("y")), V("x"), V("y")],
         ["a", "b", "x", "y"], line=262)
    case("only the least preferable choice is acceptable",
         [V("a", M(), D("a1", "a2")), V("a1", C("c1"), C("c2")), V("a2", C("c1")),
          V("b", M(), D("b1", "b2")), V("b1", C("c1"), C("c2")), V("b2", C("c1")),
          V("c", M(), D("c1", "c2")), V("c1"), V("c2")],
         ["a", "a2", "b", "b2", "c", "c2"], line=272)
    case("preferences respected with multiple dependencies per variable",
         [V("a", M(), D("x1", "x2"), D("y1", "y2")), V("x1"), V("x2"), V("y1"), V("y2")],
         ["a", "x1", "y1"], line=287)
    return {"source": "pkg/sat/solve_test.go:89-357", "cases": cases}


def errors():
    return {
        "source": "pkg/sat/solve_test.go:39-87, 359-365",
        "not_satisfiable": [
            {"name": "nil", "applied": None, "string": "constraints not satisfiable"},
            {"name": "empty", "applied": [], "string": "constraints not satisfiable"},
            {"name": "single failure", "applied": [["a", M()]],
             "string": "constraints not satisfiable: a is mandatory"},
            {"name": "multiple failures", "applied": [["a", M()], ["b", P()]],
             "string": "constraints not satisfiable: a is mandatory, b is prohibited"},
        ],
        "duplicate_identifier": {"variables": [V("a"), V("a")],
                                 "string": 'duplicate identifier "a" in input'},
        "order": [
            {"name": "mandatory", "constraint": M(), "expected": None},
            {"name": "prohibited", "constraint": P(), "expected": None},
            {"name": "dependency", "constraint": D("a", "b", "c"), "expected": ["a", "b", "c"]},
            {"name": "conflict", "constraint": C("a"), "expected": None},
        ],
    }


def testsearch():
    return {"source": "pkg/sat/search_test.go:31-106", "cases": [
        {"name": "children popped from back of deque when guess popped",
         "variables": [V("a", M(), D("c")), V("b", M()), V("c")],
         "test_returns": [0, -1], "untest_returns": [-1, -1], "result": -1, "assumptions": None},
        {"name": "candidates exhausted",
         "variables": [V("a", M(), D("x")), V("b", M(), D("y")), V("x"), V("y")],
         "test_returns": [0, 0, -1, 1], "untest_returns": [0], "result": 1,
         "assumptions": ["a", "b", "y"]},
    ]}


def readme():
    sat_vars = [V("A-v0.1.0", M(), D("C-v0.1.0")), V("B-latest", M(), D("D-latest")),
                V("C-v0.1.0"), V("D-latest")]
    unsat_vars = [V("A-v0.1.0", M(), D("C-v0.1.0")), V("B-latest", M(), D("C-v0.2.0")),
                  V("C-v0.1.0"), V("C-v0.2.0"), V("C", A(1, "C-v0.1.0", "C-v0.2.0"))]
    return {"source": "README.md:38-101 (encoding: SURVEY.md §8(d) config 1)", "cases": [
        {"name": "successful resolution", "variables": sat_vars,
         "installed": ["A-v0.1.0", "B-latest", "C-v0.1.0", "D-latest"], "error": None},
        {"name": "unsuccessful resolution", "variables": unsat_vars, "installed": None,
         "error": unsat(unsat_vars, [("A-v0.1.0", 0), ("A-v0.1.0", 1), ("B-latest", 0),
                                     ("B-latest", 1), ("C", 0)])},
    ]}


def main():
    for name, obj in [("testsolve", testsolve()), ("errors", errors()),
                      ("testsearch", testsearch()), ("readme", readme())]:
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(obj, f, indent=1, sort_keys=True)
            f.write("\n")


if __name__ == "__main__":
    main()
