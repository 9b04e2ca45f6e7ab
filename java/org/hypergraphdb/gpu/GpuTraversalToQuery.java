/*
 * GpuTraversalToQuery.java -- the GPU compilers of the traversal conditions, registered per graph
 * next to GpuAndToQuery:
 *
 *     GpuTraversalToQuery.registerAll(graph, snapshot);
 *
 * which is, spelled out (HGQueryConfiguration.addCompiler, core/.../query/HGQueryConfiguration.java:48;
 * QueryCompile.translator consults it before ToQueryMap, core/.../query/QueryCompile.java:80-87):
 *
 *     QC.addCompiler(And.class,               new GpuAndToQuery(snapshot));
 *     QC.addCompiler(SubsumedCondition.class, new GpuTraversalToQuery.Subsumed(snapshot));
 *     QC.addCompiler(SubsumesCondition.class, new GpuTraversalToQuery.Subsumes(snapshot));
 *     QC.addCompiler(BFSCondition.class,      new GpuTraversalToQuery.BFS(snapshot));
 *
 * Each mirrors the reference translator in core/.../query/cond2qry/ToQueryMap.java exactly -- the same
 * start reference, the same DefaultALGenerator flags, Integer.MAX_VALUE depth, ReturnType.targets,
 * the same QueryMetaData -- with HGGpuTraversal in place of HGBreadthFirstTraversal:
 *   hg.subsumed(G)  ToQueryMap.java:340-370  AtomTypeCondition(HGSubsumes), preceding F, succeeding T, reverse F
 *   hg.subsumes(S)  ToQueryMap.java:282-312  AtomTypeCondition(HGSubsumes), preceding F, succeeding T, reverse T
 *   hg.bfs(...)     ToQueryMap.java:313-327  BFSCondition.getTraversal (BFSCondition.java:43-45) = the
 *                   condition's own DefaultALGenerator (TraversalCondition.makeGenerator, :58-67)
 * The execute() result is TraversalBasedQuery's (TraversalBasedQuery.java:47-71): the atoms in the
 * reference's FIFO next() order, computed by hgx_bfs_sequence (order-exact, discovering links included).
 * A generator the engine does not accelerate (a sibling predicate, a link predicate that is not an
 * AtomTypeCondition) makes HGGpuTraversal build the reference HGBreadthFirstTraversal itself, and a
 * condition the reference translator would reject is passed to that translator unchanged.
 *
 * Many traversals at once: executeBatch(...) runs every start atom of a list of conditions in ONE
 * hgx_bfs_sequence call (the engine's unit of work is a batch: a single seed pays the whole fixed
 * launch and copy cost, profiles/r03d_single_latency.json).
 *
 * Executed through the JNI shim by tests/test_gpu_jni.py (fake JNIEnv); the Java itself is not
 * compiled here: no JDK exists in this build image.
 */
package org.hypergraphdb.gpu;

import java.util.ArrayList;
import java.util.List;

import org.hypergraphdb.HGException;
import org.hypergraphdb.HGHandle;
import org.hypergraphdb.HGQuery;
import org.hypergraphdb.HyperGraph;
import org.hypergraphdb.algorithms.DefaultALGenerator;
import org.hypergraphdb.algorithms.HGALGenerator;
import org.hypergraphdb.atom.HGSubsumes;
import org.hypergraphdb.query.And;
import org.hypergraphdb.query.AtomTypeCondition;
import org.hypergraphdb.query.BFSCondition;
import org.hypergraphdb.query.HGQueryCondition;
import org.hypergraphdb.query.HGQueryConfiguration;
import org.hypergraphdb.query.SubsumedCondition;
import org.hypergraphdb.query.SubsumesCondition;
import org.hypergraphdb.query.cond2qry.ConditionToQuery;
import org.hypergraphdb.query.cond2qry.QueryMetaData;
import org.hypergraphdb.query.cond2qry.ToQueryMap;
import org.hypergraphdb.query.impl.TraversalBasedQuery;
import org.hypergraphdb.util.Ref;

public abstract class GpuTraversalToQuery implements ConditionToQuery<HGHandle>
{
    protected final HGGpuSnapshot snap;

    protected GpuTraversalToQuery(HGGpuSnapshot snap) { this.snap = snap; }

    /** Registers the four GPU compilers of this package on graph's query configuration. */
    public static void registerAll(HyperGraph graph, HGGpuSnapshot snap)
    {
        HGQueryConfiguration qc = graph.getConfig().getQueryConfiguration();
        qc.addCompiler(And.class, new GpuAndToQuery(snap));
        qc.addCompiler(SubsumedCondition.class, new Subsumed(snap));
        qc.addCompiler(SubsumesCondition.class, new Subsumes(snap));
        qc.addCompiler(BFSCondition.class, new BFS(snap));
    }

    /** The reference's own translator of a condition class (the anonymous ToQueryMap entries). */
    @SuppressWarnings("unchecked")
    static ConditionToQuery<HGHandle> reference(Class<?> c)
    {
        return (ConditionToQuery<HGHandle>)ToQueryMap.getInstance().get(c);
    }

    /** The start reference of a condition, or null (the reference translator handles / rejects it). */
    abstract Ref<HGHandle> start(HGQueryCondition c);

    /** The generator the reference translator builds for a condition. */
    abstract HGALGenerator generator(HyperGraph graph, HGQueryCondition c);

    @SuppressWarnings({"unchecked", "rawtypes"})
    public HGQuery<HGHandle> getQuery(HyperGraph graph, HGQueryCondition c)
    {
        Ref<HGHandle> s = start(c);
        if (s == null)   // e.g. a value instead of a handle: the reference throws its HGException
            return reference(c.getClass()).getQuery(graph, c);
        return (HGQuery<HGHandle>)(HGQuery)new TraversalBasedQuery(
            new HGGpuTraversal(snap, s, generator(graph, c), Integer.MAX_VALUE), TraversalBasedQuery.ReturnType.targets);
    }

    /**
     * The results of many conditions of this class in one engine call: result[i] = the atoms the
     * query of conditions.get(i) returns, in its FIFO order.  All conditions must share one generator
     * (true of every subsumed / subsumes condition; BFS conditions with equal flags and predicates);
     * returns null when the generator is not accelerated (run the queries one by one).
     */
    public HGHandle[][] executeBatch(HyperGraph graph, List<? extends HGQueryCondition> conditions)
    {
        if (conditions.isEmpty()) return new HGHandle[0][];
        HGALGenerator gen = generator(graph, conditions.get(0));
        List<HGHandle> starts = new ArrayList<HGHandle>(conditions.size());
        for (HGQueryCondition c : conditions)
        {
            Ref<HGHandle> s = start(c);
            if (s == null || s.get() == null)
                throw new HGException("GPU traversal batch: condition without a start handle: " + c);
            starts.add(s.get());
        }
        return HGGpuTraversal.sequences(snap, starts.toArray(new HGHandle[starts.size()]), gen, Integer.MAX_VALUE);
    }

    /** hg.subsumed(general): the descendants of general over HGSubsumes links (ToQueryMap.java:340-370). */
    public static final class Subsumed extends GpuTraversalToQuery
    {
        public Subsumed(HGGpuSnapshot snap) { super(snap); }

        Ref<HGHandle> start(HGQueryCondition c)
        {
            SubsumedCondition sc = (SubsumedCondition)c;
            Ref<HGHandle> s = sc.getGeneralHandleReference();
            return s == null && sc.getGeneralValue() != null ? null : s;
        }

        HGALGenerator generator(HyperGraph graph, HGQueryCondition c)
        {
            return new DefaultALGenerator(graph, new AtomTypeCondition(graph.getTypeSystem().getTypeHandle(HGSubsumes.class)),
                                          null, false, true, false);
        }

        public QueryMetaData getMetaData(HyperGraph graph, HGQueryCondition c)
        {
            QueryMetaData x = QueryMetaData.MISTERY.clone(c);
            x.predicateCost = 5;
            return x;
        }
    }

    /** hg.subsumes(specific): the ancestors of specific over HGSubsumes links (ToQueryMap.java:282-312). */
    public static final class Subsumes extends GpuTraversalToQuery
    {
        public Subsumes(HGGpuSnapshot snap) { super(snap); }

        Ref<HGHandle> start(HGQueryCondition c)
        {
            SubsumesCondition sc = (SubsumesCondition)c;
            Ref<HGHandle> s = sc.getSpecificHandleReference();
            return s == null && sc.getSpecificValue() != null ? null : s;
        }

        HGALGenerator generator(HyperGraph graph, HGQueryCondition c)
        {
            return new DefaultALGenerator(graph, new AtomTypeCondition(graph.getTypeSystem().getTypeHandle(HGSubsumes.class)),
                                          null, false, true, true);
        }

        public QueryMetaData getMetaData(HyperGraph graph, HGQueryCondition c)
        {
            QueryMetaData x = QueryMetaData.MISTERY.clone(c);
            x.predicateCost = 5;
            return x;
        }
    }

    /** hg.bfs(start, linkPredicate, siblingPredicate, ...) (ToQueryMap.java:313-327). */
    public static final class BFS extends GpuTraversalToQuery
    {
        public BFS(HGGpuSnapshot snap) { super(snap); }

        Ref<HGHandle> start(HGQueryCondition c) { return ((BFSCondition)c).getStartAtomReference(); }

        HGALGenerator generator(HyperGraph graph, HGQueryCondition c) { return ((BFSCondition)c).makeGenerator(graph); }

        public QueryMetaData getMetaData(HyperGraph graph, HGQueryCondition c)
        {
            QueryMetaData x = QueryMetaData.MISTERY.clone(c);
            x.predicateCost = -1;
            x.predicateOnly = false;
            return x;
        }
    }
}
