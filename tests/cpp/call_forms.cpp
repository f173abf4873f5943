// call_forms.cpp — compile check of the drop-in boundary: the reference drivers' hot-path call forms,
// written exactly as in myapps/convection_diffusion (file:line on each), against mfem.hpp.
// tests/test_cpp_driver.py builds it with the same flags as the shipped drivers; linking it proves the
// names, signatures and ownership rules match (running it needs a GPU: the solve part is exercised by
// lib/convection_diffusion and lib/diffusion_mms).  YAML parsing (yaml-cpp) and the PETSc C API are
// outside the boundary; everything else below is the reference text.
#include "mfem.hpp"

#ifndef MFEM_USE_PETSC
#error "This driver requires MFEM built with PETSc."
#endif

#include <cmath>
#include <iostream>
#include <limits>
#include <memory>
#include <string>

using namespace std;
using namespace mfem;

namespace {

// linear_convection_diffusion_2D.cpp:129-157
void ValidateUnitSquareMesh(const ParMesh &pmesh, const double tol)
{
    double local_min[2] = {numeric_limits<double>::infinity(), numeric_limits<double>::infinity()};
    double local_max[2] = {-numeric_limits<double>::infinity(), -numeric_limits<double>::infinity()};
    for (int i = 0; i < pmesh.GetNV(); i++) {
        const double *v = pmesh.GetVertex(i);
        local_min[0] = min(local_min[0], v[0]);
        local_min[1] = min(local_min[1], v[1]);
        local_max[0] = max(local_max[0], v[0]);
        local_max[1] = max(local_max[1], v[1]);
    }
    double global_min[2] = {0.0, 0.0};
    double global_max[2] = {0.0, 0.0};
    MPI_Allreduce(local_min, global_min, 2, MPI_DOUBLE, MPI_MIN, MPI_COMM_WORLD);
    MPI_Allreduce(local_max, global_max, 2, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    MFEM_VERIFY(std::abs(global_min[0] - 0.0) <= tol && std::abs(global_max[0] - 1.0) <= tol &&
                    std::abs(global_min[1] - 0.0) <= tol && std::abs(global_max[1] - 1.0) <= tol,
                "Mesh coordinates must span approximately [0,1]x[0,1]. "
                    << "Got x=[" << global_min[0] << "," << global_max[0] << "], y=[" << global_min[1] << ","
                    << global_max[1] << "].");
}

// :159-175
class ExactSolutionCoefficient : public Coefficient {
public:
    ExactSolutionCoefficient(const int mode_n, const int mode_m) : n_(mode_n), m_(mode_m) {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        return std::sin(n_ * M_PI * x[0]) * std::sin(m_ * M_PI * x[1]);
    }

private:
    int n_;
    int m_;
};

// diffusion_mms_ale.cpp:474-502 (the metric with a fixed cofactor instead of the ALE map)
class MetricCoefficient : public MatrixCoefficient {
public:
    MetricCoefficient(double alpha, double dt) : MatrixCoefficient(2), alpha_(alpha), dt_(dt) {}
    void Eval(DenseMatrix &M, ElementTransformation &T, const IntegrationPoint &ip) override
    {
        T.Transform(ip, xhat_);
        DenseMatrix C(2, 2);
        C(0, 0) = 1.0 + 0.1 * xhat_[1];
        C(0, 1) = 0.0;
        C(1, 0) = 0.0;
        C(1, 1) = 1.0 + 0.1 * xhat_[0];
        const double J = C(0, 0) * C(1, 1);
        M.SetSize(2, 2);
        MultAAt(C, M);
        M *= alpha_ * dt_ / J;
    }

private:
    double alpha_, dt_;
    Vector xhat_;
};

}  // namespace

int main(int argc, char *argv[])
{
    Mpi::Init(argc, argv);                       // :240
    Hypre::Init();                               // :241
    const int myid = Mpi::WorldRank();           // :242

    string input_file = "Input/input_2d.yaml";  // :244-253
    string mesh_file;
    int order = 3;
    OptionsParser args(argc, argv);
    args.AddOption(&input_file, "-i", "--input", "YAML input file.");
    args.AddOption(&mesh_file, "-m", "--mesh", "Mesh file.");
    args.AddOption(&order, "-o", "--order", "Order.");
    args.Parse();
    if (!args.Good()) {
        if (myid == 0) args.PrintUsage(cout);
        return 1;
    }
    if (myid == 0) args.PrintOptions(cout);

    MFEMInitializePetsc(&argc, &argv, nullptr, NULL);  // :282

    int exit_code = 0;
    try {
        Device device("cpu");                    // :287-288
        if (myid == 0) device.Print();

        unique_ptr<Mesh> mesh = make_unique<Mesh>(mesh_file.c_str(), 1, 1);  // :290-298
        if (mesh->Dimension() != 2) throw runtime_error("The mesh must be 2D.");
        for (int l = 0; l < 0; l++) mesh->UniformRefinement();

        unique_ptr<ParMesh> pmesh = make_unique<ParMesh>(MPI_COMM_WORLD, *mesh);  // :300-305
        mesh.reset();
        for (int l = 0; l < 0; l++) pmesh->UniformRefinement();

        MFEM_VERIFY(pmesh->bdr_attributes.Size() > 0, "Mesh must define boundary attributes.");  // :307
        ValidateUnitSquareMesh(*pmesh, 1.0e-8);

        H1_FECollection fec(order, 2);           // :311-317
        ParFiniteElementSpace fespace(pmesh.get(), &fec);
        const HYPRE_BigInt global_true_dofs = fespace.GlobalTrueVSize();
        if (myid == 0) cout << "Global true dofs: " << global_true_dofs << endl;

        Array<int> ess_bdr(pmesh->bdr_attributes.Max());  // :319-322
        ess_bdr = 1;
        Array<int> ess_tdof_list;
        fespace.GetEssentialTrueDofs(ess_bdr, ess_tdof_list);

        ExactSolutionCoefficient exact_coeff(3, 3);
        Vector c_vec(2);
        c_vec[0] = 1.0;
        c_vec[1] = -2.0;
        VectorConstantCoefficient convection_coeff(c_vec);
        ConstantCoefficient kappa_coeff(0.1);
        ConstantCoefficient reaction_coeff(1.0);
        MetricCoefficient metric_coeff(0.1, 0.05);

        ParBilinearForm a(&fespace);             // :335-339
        a.AddDomainIntegrator(new DiffusionIntegrator(kappa_coeff));
        a.AddDomainIntegrator(new ConvectionIntegrator(convection_coeff));
        a.AddDomainIntegrator(new MassIntegrator(reaction_coeff));
        a.AddDomainIntegrator(new DiffusionIntegrator(metric_coeff));      // diffusion_mms_ale.cpp:1019
        a.AddDomainIntegrator(new ConvectionIntegrator(convection_coeff, -1.0));  // :1020
        a.Assemble();
        a.Finalize();

        ParLinearForm b(&fespace);               // :341-343
        b.AddDomainIntegrator(new DomainLFIntegrator(exact_coeff));
        b.Assemble();

        ParGridFunction u(&fespace);             // :345-347
        u = 0.0;
        u.ProjectBdrCoefficient(exact_coeff, ess_bdr);

        Vector rhs_local(fespace.GetVSize());     // diffusion_mms.cpp:421,430,437
        a.Mult(u, rhs_local);
        rhs_local.Add(0.05, b);

        OperatorHandle Ah(Operator::Hypre_ParCSR);  // :349-351
        Vector X, B;
        a.FormLinearSystem(ess_tdof_list, u, b, Ah, X, B);

        const int true_size = fespace.TrueVSize();  // :353-375
        const bool all_essential = (ess_tdof_list.Size() == true_size);
        if (!all_essential) {
            HypreParMatrix *A_true = Ah.As<HypreParMatrix>();
            MFEM_VERIFY(A_true != nullptr, "Expected HypreParMatrix from FormLinearSystem.");
            PetscParMatrix A_petsc(MPI_COMM_WORLD, A_true, Operator::PETSC_MATAIJ);
            PetscLinearSolver solver(A_petsc);
            solver.SetPrintLevel(0);
            solver.Mult(B, X);
            MFEM_VERIFY(solver.GetConverged(), "PETSc solver did not converge. Iterations="
                                                   << solver.GetNumIterations() << ", residual=" << solver.GetFinalNorm());
            PetscParMatrix A_petsc2(A_true, Operator::PETSC_MATAIJ);  // diffusion_mms.cpp:449
            PetscLinearSolver solver2(A_petsc2);
            solver2.SetRelTol(1e-10);                                // diffusion_mms_ale.cpp:693-696
            solver2.SetAbsTol(0.0);
            solver2.SetMaxIter(400);
            solver2.SetPrintLevel(0);
            solver2.Mult(B, X);
        }

        a.RecoverFEMSolution(X, b, u);           // :377

        ParGridFunction u_exact(&fespace);       // :379-381
        u_exact = 0.0;
        u_exact.ProjectCoefficient(exact_coeff);
        ParGridFunction u_error(&fespace);       // diffusion_mms.cpp:375-383
        subtract(u, u_exact, u_error);
        const double local_linf = u_error.Normlinf();
        double linf_err = 0.0;
        MPI_Allreduce(&local_linf, &linf_err, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);

        int order_quad = std::max(2, 2 * order + 3);  // :383-392
        const IntegrationRule *irs[Geometry::NumGeom];
        for (int g = 0; g < Geometry::NumGeom; g++) irs[g] = &IntRules.Get(g, order_quad);
        const double abs_l2 = u.ComputeL2Error(exact_coeff, irs);
        const double exact_l2 = ComputeGlobalLpNorm(2, exact_coeff, *pmesh, irs);
        const double rel_l2 = (exact_l2 > 1.0e-14) ? abs_l2 / exact_l2 : 0.0;
        ConstantCoefficient j_coeff(1.0);
        const double l2_w = u.ComputeLpError(2.0, exact_coeff, &j_coeff, irs);  // diffusion_mms_ale.cpp:924
        if (myid == 0) cout << "L2 error (absolute): " << abs_l2 << " relative " << rel_l2 << " " << l2_w << endl;

        const bool save_paraview = false;        // :421-433
        if (save_paraview) {
            ParaViewDataCollection paraview_dc("convection_diffusion_2D", pmesh.get());
            paraview_dc.SetPrefixPath("ParaView");
            paraview_dc.SetLevelsOfDetail(order);
            paraview_dc.SetDataFormat(VTKFormat::BINARY);
            paraview_dc.SetHighOrderOutput(true);
            paraview_dc.RegisterField("u", &u);
            paraview_dc.SetCycle(0);
            paraview_dc.SetTime(0.0);
            paraview_dc.Save();
        }
    } catch (const exception &e) {               // :435-442
        if (myid == 0) cerr << "Error: " << e.what() << endl;
        exit_code = 3;
    }

    MFEMFinalizePetsc();                         // :444
    return exit_code;
}
