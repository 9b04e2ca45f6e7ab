/*
 * GpuAndToQuery.java -- the GPU compiler of conjunctive queries, registered per graph:
 *
 *     graph.getConfig().getQueryConfiguration().addCompiler(And.class, new GpuAndToQuery(snapshot));
 *
 * QueryCompile.translator consults this registry before the global ToQueryMap
 * (core/.../query/QueryCompile.java:80-87, HGQueryConfiguration.java:48), so every And the
 * ExpressionBasedQuery pipeline produces (after preprocess / expand / toDNF, ExpressionBasedQuery.java:
 * 603-875: orderedLink(x, _, y) has become And{..., incident(x), incident(y), orderedLink(...)}) comes
 * here first.  The shape {AtomTypeCondition?, IncidentCondition*, OrderedLinkCondition?} runs on the
 * GPU (hgx_pattern_batch_packed: the zig-zag intersection of ZigZagIntersectionResult + the
 * PredicateBasedFilter(OrderedLinkCondition) of AndToQuery.java:102-306, in one batch); anything else
 * -- and an engine status HGX_E_UNSUPPORTED -- is delegated to the reference's own new AndToQuery().
 *
 * Variables (Ref / Var targets, TC/query/QueryCompilation.java:35-73) are resolved when the query
 * executes, in the executing thread, so one compiled query serves many threads
 * (QueryCompilation.java:76-122); the engine's entry points are thread-safe.
 *
 * UNVERIFIED: written against the cited reference interfaces; no JDK exists in this build image.
 */
package org.hypergraphdb.gpu;

import java.util.ArrayList;
import java.util.List;

import org.hypergraphdb.HGHandle;
import org.hypergraphdb.HGQuery;
import org.hypergraphdb.HGRandomAccessResult;
import org.hypergraphdb.HGSearchResult;
import org.hypergraphdb.HyperGraph;
import org.hypergraphdb.query.And;
import org.hypergraphdb.query.AtomTypeCondition;
import org.hypergraphdb.query.HGQueryCondition;
import org.hypergraphdb.query.IncidentCondition;
import org.hypergraphdb.query.OrderedLinkCondition;
import org.hypergraphdb.query.cond2qry.AndToQuery;
import org.hypergraphdb.query.cond2qry.ConditionToQuery;
import org.hypergraphdb.query.cond2qry.QueryMetaData;
import org.hypergraphdb.util.ArrayBasedSet;
import org.hypergraphdb.util.Ref;

public class GpuAndToQuery implements ConditionToQuery<HGHandle>
{
    private final HGGpuSnapshot snap;
    private final AndToQuery<HGHandle> cpu = new AndToQuery<HGHandle>();

    public GpuAndToQuery(HGGpuSnapshot snap) { this.snap = snap; }

    /** The same metadata as AndToQuery (ORACCESS over the same sub-conditions, AndToQuery.java:73-100). */
    public QueryMetaData getMetaData(HyperGraph graph, HGQueryCondition condition)
    {
        return cpu.getMetaData(graph, condition);
    }

    /** The recognised shape: references, resolved at execution time. */
    static final class Shape
    {
        AtomTypeCondition type;                         // <= 1
        final List<Ref<HGHandle>> incident = new ArrayList<Ref<HGHandle>>();
        Ref<HGHandle>[] ordered;                        // <= 1 OrderedLinkCondition

        static Shape of(And and)
        {
            Shape s = new Shape();
            for (HGQueryCondition c : and)
            {
                if (c instanceof AtomTypeCondition && s.type == null) s.type = (AtomTypeCondition)c;
                else if (c instanceof IncidentCondition) s.incident.add(((IncidentCondition)c).getTargetRef());
                else if (c instanceof OrderedLinkCondition && s.ordered == null)
                    s.ordered = ((OrderedLinkCondition)c).getTargets();
                else return null;   // another condition (or a second type / orderedLink): the CPU compiler
            }
            if (s.incident.isEmpty() && s.ordered == null) return null;   // no incidence anchor
            return s;
        }
    }

    public HGQuery<HGHandle> getQuery(final HyperGraph graph, final HGQueryCondition condition)
    {
        final And and = (And)condition;
        final Shape shape = and.isEmpty() ? null : Shape.of(and);
        if (shape == null)
            return cpu.getQuery(graph, condition);
        HGQuery<HGHandle> q = new HGQuery<HGHandle>()
        {
            public HGSearchResult<HGHandle> execute()
            {
                try
                {
                    return result(executeBatch(graph, new Shape[] {shape})[0]);
                }
                catch (UnsupportedOperationException e)
                {
                    return cpu.getQuery(graph, condition).execute();
                }
            }
        };
        q.setHyperGraph(graph);
        return q;
    }

    /** Sorted handles as a random-access result (nested intersections goTo into it, ArrayBasedSet.java:457-543). */
    static HGRandomAccessResult<HGHandle> result(HGHandle[] sorted)
    {
        return new ArrayBasedSet<HGHandle>(sorted).getSearchResult();
    }

    /**
     * Many expanded And queries in one engine call (hgx_pattern_batch_packed): result[q] = the links
     * of query q in handle order.  Throws UnsupportedOperationException when one of them is not of
     * the accelerated shape (the caller runs those through the reference compiler).
     */
    public HGHandle[][] executeBatch(HyperGraph graph, List<And> queries)
    {
        Shape[] shapes = new Shape[queries.size()];
        for (int q = 0; q < shapes.length; q++)
            if ((shapes[q] = Shape.of(queries.get(q))) == null)
                throw new UnsupportedOperationException("query " + q + " is not {type?, incident*, orderedLink?}");
        return executeBatch(graph, shapes);
    }

    HGHandle[][] executeBatch(HyperGraph graph, Shape[] shapes)
    {
        snap.sync();
        int n = shapes.length;
        int[] type = new int[n], hasOrdered = new int[n];
        long[] incOff = new long[n + 1], patOff = new long[n + 1];
        List<Integer> inc = new ArrayList<Integer>(), pat = new ArrayList<Integer>();
        boolean[] empty = new boolean[n];
        HGHandle any = graph.getHandleFactory().anyHandle();
        for (int q = 0; q < n; q++)
        {
            Shape s = shapes[q];
            type[q] = Hgx.NO_TYPE;
            if (s.type != null)
            {
                HGHandle th = s.type.getTypeHandle(graph);
                int k = th == null ? -1 : snap.typeKeyOrNone(th);
                if (k < 0) empty[q] = true;   // no stored link has this type: the result is empty
                type[q] = Math.max(k, 0);
            }
            for (Ref<HGHandle> r : s.incident)
                inc.add(snap.rank(r.get()));
            incOff[q + 1] = inc.size();
            if (s.ordered != null)
            {
                hasOrdered[q] = 1;
                for (Ref<HGHandle> r : s.ordered)
                {
                    HGHandle h = r.get();
                    boolean isAny = h == null || h == HGQuery.hg.anyHandle() || h.equals(any);   // hg.anyHandle()
                    pat.add(isAny ? Hgx.ANY_HANDLE : snap.rank(h));
                }
            }
            patOff[q + 1] = pat.size();
        }
        long res = Hgx.patternBatch(snap.native_(), type, incOff, toArray(inc), hasOrdered, patOff, toArray(pat));
        try
        {
            long[] off = Hgx.queryOffsets(res);
            int[] ids = Hgx.queryIds(res);
            HGHandle[][] out = new HGHandle[n][];
            for (int q = 0; q < n; q++)
            {
                int a = (int)off[q], b = empty[q] ? a : (int)off[q + 1];
                int[] part = new int[b - a];
                System.arraycopy(ids, a, part, 0, b - a);
                out[q] = snap.handles(part);
            }
            return out;
        }
        finally
        {
            Hgx.queryFree(res);
        }
    }

    private static int[] toArray(List<Integer> v)
    {
        int[] a = new int[v.size()];
        for (int i = 0; i < a.length; i++) a[i] = v.get(i);
        return a;
    }
}
