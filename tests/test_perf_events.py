"""PerfEvents of Decision's pending updates (Decision.cpp:35-95, aux SURVEY
§5) and the LsdbUtil helpers (LsdbUtil.cpp:40-128), host only. Cases follow
the reference's own tests: DecisionTest.cpp:3282-3305 (DecisionPendingUpdates
perfEvents) and UtilTest.cpp:475-546 (sprintPerfEvents,
getTotalPerfEventsDuration, getDurationBetweenPerfEvents); the publication
path carries each database's events (Decision.cpp:739, 779)."""
import pytest

pytestmark = pytest.mark.filterwarnings("ignore")


@pytest.fixture(scope="module")
def M(host_module):
    return host_module


def test_pending_updates_perf_events(M):
    """DecisionTest.cpp:3282-3305: an update without events starts the
    batch's list with DECISION_RECEIVED; an update whose events are older
    displaces it (EARLIER, then DECISION_RECEIVED)."""
    u = M.DecisionPendingUpdates("node1")
    u.applyLinkStateChange("node2", {})
    ev = u.perfEvents()
    assert len(ev) == 1 and ev[0][1] == "DECISION_RECEIVED" and ev[0][0] == "node1"
    u.applyPrefixStateChange([], [("node3", "EARLIER", 1)])
    ev = u.perfEvents()
    assert [e[1] for e in ev] == ["EARLIER", "DECISION_RECEIVED"]
    # a newer list does not displace the older one
    u.applyPrefixStateChange([], [("node4", "LATER", ev[-1][2] + 10_000)])
    assert [e[1] for e in u.perfEvents()] == ["EARLIER", "DECISION_RECEIVED"]
    assert u.getCount() == 3
    u.addEvent("DECISION_DEBOUNCE")
    d, err = M.getDurationBetweenPerfEvents(u.perfEvents(), "DECISION_RECEIVED",
                                            "DECISION_DEBOUNCE")
    assert err is None and d >= 0
    out = u.moveOutEvents()
    assert [e[1] for e in out] == ["EARLIER", "DECISION_RECEIVED", "DECISION_DEBOUNCE"]
    assert u.perfEvents() is None
    u.addEvent("ROUTE_UPDATE")  # no list: nothing recorded (Decision.cpp:62-67)
    assert u.perfEvents() is None
    u.reset()
    assert u.getCount() == 0 and u.perfEvents() is None


def test_perf_event_helpers(M):
    """UtilTest.cpp:475-546."""
    assert M.sprintPerfEvents([]) == []
    ev = M.addPerfEvent([], "node1", "LINK_UP")
    ev = M.addPerfEvent(ev, "node2", "LINK_DOWN")
    s = M.sprintPerfEvents(ev)
    assert len(s) == 2
    assert s[0].startswith("node: node1, event: LINK_UP")
    assert s[1].startswith("node: node2, event: LINK_DOWN")
    assert M.getTotalPerfEventsDuration([]) == 0
    ev = [("node1", "LINK_UP", 100), ("node1", "DECISION_RECVD", 200),
          ("node1", "SPF_CALCULATE", 300)]
    assert M.getTotalPerfEventsDuration(ev) == 200
    assert M.getDurationBetweenPerfEvents([], "LINK_UP", "SPF_CALCULATE")[0] is None
    assert M.getDurationBetweenPerfEvents(ev, "LINK_UP", "SPF_CALCULATE") == (200, None)
    assert M.getDurationBetweenPerfEvents(ev, "DECISION_RECVD", "SPF_CALCULATE") == (100, None)
    for a, b in (("NO_SUCH_NAME", "SPF_CALCULATE"), ("SPF_CALCULATE", "DECISION_RECVD"),
                 ("DECISION_RECVD", "NO_SUCH_NAME")):
        d, err = M.getDurationBetweenPerfEvents(ev, a, b)
        assert d is None and err


def test_publication_carries_perf_events(M):
    """An adjacency database's perfEvents (Types.thrift:250, field 5) survive
    the codec and reach the pending updates through the publication path;
    the oldest list wins the batch."""
    adj = {"thisNodeName": "n1", "area": "0", "nodeLabel": 0,
           "adjacencies": [], "perfEvents": [("n1", "ADJ_DB_UPDATED", 5)]}
    raw = M.encodeAdjDb(adj)
    back = M.decodeAdjDb(raw)
    assert back["perfEvents"] == [("n1", "ADJ_DB_UPDATED", 5)]
    adj2 = dict(adj, thisNodeName="n2", perfEvents=[("n2", "ADJ_DB_UPDATED", 3)])
    ing = M.LsdbIngest("me", {"0"})
    ls = M.LinkState("0", "me")
    ps = M.PrefixState()
    for key, d in (("adj:n1", adj), ("adj:n2", adj2)):
        u = ing.updateKeyInLsdb("0", ls, ps, key, M.encodeAdjDb(d))
        assert u["perfEvents"] == d["perfEvents"]
    # the publication path: n1's list (ts 5), then n2's older one (ts 3)
    als = M.AreaLinkStates()
    pending = M.DecisionPendingUpdates("me")
    ing.processPublicationKeyVals("0", als, M.PrefixState(),
                                  [("adj:n1", M.encodeAdjDb(adj)), ("adj:n2", M.encodeAdjDb(adj2))],
                                  [], pending)
    ev = pending.perfEvents()
    assert [e[:2] for e in ev] == [("n2", "ADJ_DB_UPDATED"), ("me", "DECISION_RECEIVED")]
    assert pending.getCount() == 2
