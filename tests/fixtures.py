"""Helpers shared by the tests: golden fixtures -> problems, result mapping."""
import json
import os

from oracle import lower_ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KIND = {"mandatory": 1, "prohibited": 2, "dependency": 3, "conflict": 4, "atmost": 5}


def load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


def to_problem(variables):
    """Fixture variables -> lower_ref problem (bytes identifiers)."""
    out = []
    for v in variables:
        cons = []
        for c in v["constraints"]:
            cons.append((KIND[c["kind"]], c.get("n", 0), [i.encode() for i in c.get("ids", [])]))
        out.append((v["id"].encode(), cons))
    return out


def cstr(subject, c):
    """Constraint.String(subject), constraints.go:57,81,108-114,145,173-177."""
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
    return "%s permits at most %d of %s" % (subject, c["n"], ", ".join(c["ids"]))


def sorted_applied(variables, applied):
    """applied: [(var index, constraint index)] -> test-sorted [{'var', 'constraint'}]
    (solve_test.go:316-343: by identifier, then constraint position)."""
    items = [(variables[vi]["id"], ci) for vi, ci in applied]
    items.sort(key=lambda t: (t[0].encode(), t[1]))
    return [{"var": v, "constraint": ci} for v, ci in items]


def not_satisfiable_string(variables, applied_sorted):
    by = {v["id"]: v for v in variables}
    if not applied_sorted:
        return "constraints not satisfiable"
    return "constraints not satisfiable: " + ", ".join(
        cstr(a["var"], by[a["var"]]["constraints"][a["constraint"]]) for a in applied_sorted)


def wire_problem_variables(w, p):
    """Problem p of a generated wire batch (_lib.generate) as sat Variables."""
    from deppy_amd import sat
    from tests.test_lowering import V

    so, sb = w["str_off"], w["str_bytes"].tobytes()

    def s(i):
        return sb[so[i]:so[i + 1]].decode()

    out = []
    for v in range(int(w["prob_var_off"][p]), int(w["prob_var_off"][p + 1])):
        cons = []
        for c in range(int(w["var_con_off"][v]), int(w["var_con_off"][v + 1])):
            k, n = int(w["con_kind"][c]), int(w["con_n"][c])
            args = [s(int(a)) for a in w["con_arg"][w["con_arg_off"][c]:w["con_arg_off"][c + 1]]]
            if k == 1:
                cons.append(sat.Mandatory())
            elif k == 2:
                cons.append(sat.Prohibited())
            elif k == 3:
                cons.append(sat.Dependency(*args))
            elif k == 4:
                cons.append(sat.Conflict(args[0]))
            else:
                cons.append(sat.AtMost(n, *args))
        out.append(V(s(int(w["var_id"][v])), *cons))
    return out
