"""CPU tests of the Flask endpoint's request handling (web/__init__.py mirrors the reference's
GET /?cube_name=&num_recs=&root=): the recommend call itself is stubbed (it needs the GPU and the
network), so this checks parameters, defaults, error strings and the JSON result."""
import pytest

flask = pytest.importorskip('flask')


def test_endpoint_parameters_and_json(monkeypatch):
    import web
    calls = []

    def fake(cube_name, amount, root):
        calls.append((cube_name, amount, root))
        return {'additions': {'b card': 0.75, 'a card': 0.5}, 'cuts': {'c card': 0.25}}
    monkeypatch.setattr(web, 'get_ml_recommend', fake)
    c = web.app.test_client()
    r = c.get('/?cube_name=mycube')
    assert r.status_code == 200
    assert r.get_json() == {'additions': {'b card': 0.75, 'a card': 0.5}, 'cuts': {'c card': 0.25}}
    assert calls[-1] == ('mycube', 30000, 'https://www.cubecobra.com')
    c.get('/?cube_name=x&num_recs=12&root=http://local')
    assert calls[-1] == ('x', 12, 'http://local')
    assert c.get('/').get_data(as_text=True) == 'Need cube_name and num_recs as parameters!'
    assert c.get('/?cube_name=x&num_recs=ten').get_data(as_text=True) == 'num_recs needs to be an integer!'
    assert len(calls) == 2
