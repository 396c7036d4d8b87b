"""RAG lab: retriever behaviour (TF-IDF + fallback), prompt format, end-to-end CLI on CPU."""
from mift.apps.rag import Retriever, build_prompt, main, overlap_score


def test_retrievers_rank_relevant_doc_first():
    docs = ["oil prices rise as opec cuts output", "team wins the football championship final",
            "new computer chip doubles speed", "stocks fall on wall street"]
    for fb in (False, True):
        r = Retriever(docs, force_fallback=fb)
        assert r.search("who won the football championship", k=2)[0][0] == 1
        assert r.search("computer chip speed", k=1)[0][0] == 2
    assert overlap_score("a b", "") == 0.0


def test_prompt_format():
    p = build_prompt("Q?", ["p1", "p2"])
    assert p.startswith("Answer the question concisely using the context.\nContext:\n- p1\n\n- p2")
    assert p.endswith("Question: Q?\nAnswer:")


def test_rag_cli_end_to_end(tmp_path, monkeypatch):
    monkeypatch.setenv("MIFT_DEVICE", "cpu")
    monkeypatch.setenv("MIFT_AGNEWS", "synthetic")
    q = tmp_path / "q.txt"
    q.write_text("market profit bank\nleague coach season\n")
    res = main(["--dry_run", "--subset", "200", "--queries_file", str(q), "--max_new_tokens", "4",
                "--generator", "t5-tiny"])
    assert len(res) == 2 and all(isinstance(a, str) for _, a, _ in res)
    assert len(res[0][2]) == 3
